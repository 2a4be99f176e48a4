"""Python host mirror of the checksum engine (plumbing over libicsum.so).

The reference's interface for this path is the C++ header surface of
util/tools/checksum.h, util/ipv4_header, util/tcp_segment and util/tcp_over_ip
(SURVEY.md §8b); its C++ mirror lives in csrc/host/.  This module exposes the
same batch entry points to Python for tests and bench.py.  Device memory and
streams come from PyTorch (plumbing only); every byte of arithmetic runs in
the HIP kernels behind the C-ABI.  There is no fallback: a missing library or
GPU raises.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check

MODE_COMPUTE, MODE_VERIFY, MODE_PATCH = _lib.ICS_MODE_COMPUTE, _lib.ICS_MODE_VERIFY, _lib.ICS_MODE_PATCH
ST_ACCEPT = _lib.ICS_ST_ACCEPT
TCP_FIN, TCP_SYN, TCP_RST, TCP_ACK = _lib.ICS_TCP_FIN, _lib.ICS_TCP_SYN, _lib.ICS_TCP_RST, _lib.ICS_TCP_ACK

# struct ics_tcp_msg (include/icsum.h) as a numpy record
TCP_MSG_DTYPE = np.dtype([("src", "<u4"), ("dst", "<u4"), ("seqno", "<u4"), ("ackno", "<u4"),
                          ("src_port", "<u2"), ("dst_port", "<u2"), ("window", "<u2"), ("flags", "u1"),
                          ("ttl", "u1"), ("id", "<u2"), ("reserved", "<u2")])
assert TCP_MSG_DTYPE.itemsize == 28


def _ptr(t):
    if t is None:
        return None
    if isinstance(t, np.ndarray):
        return t.ctypes.data
    return t.data_ptr()


def _stream(stream, device):
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)


def _count(n, offsets, data, stride):
    """Segments of a batch: n when given, else from the offsets (n + 1
    entries), else from a positive fixed stride; a fixed-stride batch with no
    stride and no n is an error (not one segment per byte)."""
    if n is not None:
        return int(n)
    if offsets is not None:
        return offsets.numel() - 1
    if not stride or stride <= 0:
        raise ValueError("batch without n, offsets or a positive stride")
    return data.numel() // stride


class Engine:
    """One engine context bound to one GPU (ics_create / ics_destroy)."""

    def __init__(self, device=0, debug=False):
        """debug=True: the bounds-checked build (libicsum_debug.so)."""
        self.lib = _lib.load(_lib.DEBUG_LIB_PATH if debug else None)
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        ctx = ctypes.c_void_p()
        self._check(self.lib.ics_create(self.device.index or 0, ctypes.byref(ctx)))
        self.ctx = ctx

    def _check(self, rc):
        return check(rc, self.lib)

    def set_binning(self, mode):
        """Dispatch of offsets batches: _lib.ICS_BINNING_AUTO / SINGLE / BINNED
        (ics_set_binning)."""
        self._check(self.lib.ics_set_binning(self.ctx, int(mode)))

    def set_tick_server(self, idle_us):
        """ics_set_tick_server: idle_us > 0 keeps a resident kernel that takes
        the zero-copy *_host calls of <= 16 x blocks segments without a launch
        (it leaves after idle_us without a call); 0 stops it."""
        self._check(self.lib.ics_set_tick_server(self.ctx, int(idle_us)))

    def set_tick_server_blocks(self, blocks):
        """ics_set_tick_server_blocks: the resident server's blocks, 1..8
        (default 4), 16 segments per block."""
        self._check(self.lib.ics_set_tick_server_blocks(self.ctx, int(blocks)))

    def dispatch_info(self):
        """ics_dispatch_info: {'plan_hits', 'plan_misses', 'plan_requests',
        'kernel' (name of the last call's main launch), 'lps', 'unroll', 'plan',
        'host_zero_copy', 'host_dma_chunks' (the *_host pipeline's counters)}."""
        d = _lib.DispatchInfo()
        self._check(self.lib.ics_dispatch_info(self.ctx, ctypes.byref(d)))
        return {"plan_hits": d.plan_hits, "plan_misses": d.plan_misses, "plan_requests": d.plan_requests,
                "kernel": _lib.KERNELS.get(d.last_kernel), "lps": d.last_lps, "unroll": d.last_unroll,
                "plan": d.last_plan, "host_zero_copy": d.host_zero_copy, "host_dma_chunks": d.host_dma_chunks}

    def close(self):
        if self.ctx:
            self.lib.ics_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- a1-a4 -----------------------------------------------------------
    def checksum_batch(self, data, n=None, offsets=None, stride=0, seg_len=0, init=None, out=None,
                       stream=None):
        """u16 InternetChecksum{init_i}.add(segment_i).value() for every segment."""
        n = _count(n, offsets, data, stride)
        if out is None:
            out = torch.empty(n, dtype=torch.int16, device=self.device)
        self._check(self.lib.ics_checksum_batch(self.ctx, _ptr(data), _ptr(offsets), stride, seg_len,
                                          _ptr(init), _ptr(out), n, _stream(stream, self.device)))
        return out

    def sum_batch(self, data, n=None, offsets=None, stride=0, seg_len=0, init=None, odd=None,
                  out=None, stream=None):
        """Unfolded uint32 sum_ after add(segment_i) with parity odd_i (add() chains)."""
        n = _count(n, offsets, data, stride)
        if out is None:
            out = torch.empty(n, dtype=torch.int32, device=self.device)
        self._check(self.lib.ics_sum_batch(self.ctx, _ptr(data), _ptr(offsets), stride, seg_len, _ptr(init),
                                     _ptr(odd), _ptr(out), n, _stream(stream, self.device)))
        return out

    def fold_batch(self, sums, out=None, stream=None):
        n = sums.numel()
        if out is None:
            out = torch.empty(n, dtype=torch.int16, device=self.device)
        self._check(self.lib.ics_fold_batch(self.ctx, _ptr(sums), _ptr(out), n, _stream(stream, self.device)))
        return out

    def checksum_batchv(self, batches, stream=None):
        """ics_checksum_batchv: several checksum batches in one launch per
        kernel shape.  `batches`: dicts with keys data, n, offsets, stride,
        seg_len, init, out (out allocated when absent); returns the outs."""
        arr = (_lib.SegBatch * max(1, len(batches)))()
        outs = []
        for j, b in enumerate(batches):
            offsets = b.get("offsets")
            n = _count(b.get("n"), offsets, b["data"], b.get("stride", 0))
            out = b.get("out")
            if out is None:
                out = torch.empty(n, dtype=torch.int16, device=self.device)
            arr[j] = _lib.SegBatch(_ptr(b["data"]), _ptr(offsets), b.get("stride", 0), b.get("seg_len", 0), n,
                                   _ptr(b.get("init")), _ptr(out))
            outs.append(out)
        self._check(self.lib.ics_checksum_batchv(self.ctx, arr, len(batches), _stream(stream, self.device)))
        return outs

    def ipv4_tcp_batchv(self, batches, mode, stream=None):
        """ics_ipv4_tcp_batchv: dicts with keys dgrams, n, offsets, stride,
        dgram_len, ip_ck, tcp_ck, status (outputs allocated when absent);
        returns [(ip_ck, tcp_ck, status), ...]."""
        arr = (_lib.DgramBatch * max(1, len(batches)))()
        outs = []
        for j, b in enumerate(batches):
            offsets = b.get("offsets")
            n = _count(b.get("n"), offsets, b["dgrams"], b.get("stride", 0))
            mk = lambda dt: torch.empty(n, dtype=dt, device=self.device)  # noqa: E731
            o = tuple(b.get(k) if b.get(k) is not None else mk(dt)
                      for k, dt in (("ip_ck", torch.int16), ("tcp_ck", torch.int16), ("status", torch.uint8)))
            arr[j] = _lib.DgramBatch(_ptr(b["dgrams"]), _ptr(offsets), b.get("stride", 0), b.get("dgram_len", 0), n,
                                     _ptr(o[0]), _ptr(o[1]), _ptr(o[2]))
            outs.append(o)
        self._check(self.lib.ics_ipv4_tcp_batchv(self.ctx, arr, len(batches), mode, _stream(stream, self.device)))
        return outs

    # ---- fused IPv4 + TCP --------------------------------------------------
    def ipv4_tcp_batch(self, dgrams, mode, n=None, offsets=None, stride=0, dgram_len=0,
                       ip_ck=None, tcp_ck=None, status=None, stream=None):
        n = _count(n, offsets, dgrams, stride)
        mk = lambda dt: torch.empty(n, dtype=dt, device=self.device)  # noqa: E731
        ip_ck = mk(torch.int16) if ip_ck is None else ip_ck
        tcp_ck = mk(torch.int16) if tcp_ck is None else tcp_ck
        status = mk(torch.uint8) if status is None else status
        self._check(self.lib.ics_ipv4_tcp_batch(self.ctx, _ptr(dgrams), _ptr(offsets), stride, dgram_len, n,
                                          mode, _ptr(ip_ck), _ptr(tcp_ck), _ptr(status),
                                          _stream(stream, self.device)))
        return ip_ck, tcp_ck, status

    # ---- device-side wrap (wrap_tcp_in_ip, tcp_over_ip.cpp:69-88) ----------
    def tcp_wrap_batch(self, dgrams, msgs, n=None, offsets=None, stride=0, dgram_len=0, ip_ck=None,
                       tcp_ck=None, stream=None):
        """Headers + both checksums of every datagram written in place on the
        device; `msgs` is a device tensor holding n ics_tcp_msg records."""
        n = _count(n, offsets, dgrams, stride)
        self._check(self.lib.ics_tcp_wrap_batch(self.ctx, _ptr(dgrams), _ptr(offsets), stride, dgram_len, n,
                                          _ptr(msgs), _ptr(ip_ck), _ptr(tcp_ck), _stream(stream, self.device)))
        return dgrams

    def tcp_wrap_headers(self, payloads, msgs, hdrs, n=None, offsets=None, stride=0, payload_len=0, ip_ck=None,
                         tcp_ck=None, stream=None):
        """Payload-only batch; the 40 header bytes of datagram i go to hdrs[40 i:]."""
        n = _count(n, offsets, payloads, stride)
        self._check(self.lib.ics_tcp_wrap_headers(self.ctx, _ptr(payloads), _ptr(offsets), stride, payload_len, n,
                                                  _ptr(msgs), _ptr(hdrs), _ptr(ip_ck), _ptr(tcp_ck),
                                                  _stream(stream, self.device)))
        return hdrs

    def tcp_wrap_headers_host(self, payloads, msgs, n, offsets=None, stride=0, payload_len=0):
        msgs = np.ascontiguousarray(msgs, dtype=TCP_MSG_DTYPE)
        hdrs = np.empty(n * 40, dtype=np.uint8)
        self._check(self.lib.ics_tcp_wrap_headers_host(self.ctx, _ptr(payloads), _ptr(offsets), stride, payload_len,
                                                       n, msgs.ctypes.data, hdrs.ctypes.data))
        return hdrs

    def tcp_wrap_batch_host(self, dgrams, msgs, n, offsets=None, stride=0, dgram_len=0):
        """The same on host memory (numpy uint8 datagrams, TCP_MSG_DTYPE records)."""
        msgs = np.ascontiguousarray(msgs, dtype=TCP_MSG_DTYPE)
        self._check(self.lib.ics_tcp_wrap_batch_host(self.ctx, _ptr(dgrams), _ptr(offsets), stride, dgram_len, n,
                                               msgs.ctypes.data))
        return dgrams

    def router_ttl_batch(self, dgrams, n=None, offsets=None, stride=0, dgram_len=0, status=None,
                         stream=None):
        n = _count(n, offsets, dgrams, stride)
        status = torch.empty(n, dtype=torch.uint8, device=self.device) if status is None else status
        self._check(self.lib.ics_router_ttl_batch(self.ctx, _ptr(dgrams), _ptr(offsets), stride, dgram_len, n,
                                            _ptr(status), _stream(stream, self.device)))
        return status

    def router_ttl_headers(self, dgrams, n=None, offsets=None, stride=0, dgram_len=0, hdrs=None, status=None,
                           stream=None):
        """The router step with the forwarded 20-byte headers into `hdrs`
        (allocated when absent); the datagrams are only read.  Returns
        (hdrs, status)."""
        n = _count(n, offsets, dgrams, stride)
        hdrs = torch.empty(n * 20, dtype=torch.uint8, device=self.device) if hdrs is None else hdrs
        status = torch.empty(n, dtype=torch.uint8, device=self.device) if status is None else status
        self._check(self.lib.ics_router_ttl_headers(self.ctx, _ptr(dgrams), _ptr(offsets), stride, dgram_len, n,
                                                    _ptr(hdrs), _ptr(status), _stream(stream, self.device)))
        return hdrs, status

    # ---- host-memory (PCIe-inclusive) variants -----------------------------
    def checksum_batch_host(self, data, n, offsets=None, stride=0, seg_len=0, init=None):
        out = np.empty(n, dtype=np.uint16)
        self._check(self.lib.ics_checksum_batch_host(self.ctx, _ptr(data), _ptr(offsets), stride, seg_len,
                                               _ptr(init), _ptr(out), n))
        return out

    def ipv4_tcp_batch_host(self, dgrams, n, mode, offsets=None, stride=0, dgram_len=0):
        ip = np.empty(n, dtype=np.uint16)
        tcp = np.empty(n, dtype=np.uint16)
        st = np.empty(n, dtype=np.uint8)
        self._check(self.lib.ics_ipv4_tcp_batch_host(self.ctx, _ptr(dgrams), _ptr(offsets), stride, dgram_len,
                                               n, mode, _ptr(ip), _ptr(tcp), _ptr(st)))
        return ip, tcp, st

    # ---- synthetic workloads (include/icsum_workload.h) -------------------
    def fill_bytes(self, t, seed, pos0=0, stream=None):
        self._check(self.lib.icsw_fill_bytes(self.ctx, _ptr(t), t.numel() * t.element_size(), seed, pos0,
                                       _stream(stream, self.device)))
        return t

    def pseudo_inits(self, n, seed, offsets=None, seg_len=0, index0=0, out=None, stream=None):
        out = torch.empty(n, dtype=torch.int32, device=self.device) if out is None else out
        self._check(self.lib.icsw_pseudo_inits(self.ctx, _ptr(out), _ptr(offsets), seg_len, n, seed, index0,
                                         _stream(stream, self.device)))
        return out

    def ipv4_tcp_headers(self, dgrams, n, stride, dgram_len, seed, index0=0, stream=None):
        self._check(self.lib.icsw_ipv4_tcp_headers(self.ctx, _ptr(dgrams), stride, dgram_len, n, seed, index0,
                                             _stream(stream, self.device)))
        return dgrams


def device_count():
    c = ctypes.c_int()
    check(_lib.load().ics_device_count(ctypes.byref(c)))
    return c.value


def mixed_offsets(n, seed):
    """Packed uint64 offsets (n+1) of the mixed-length workload (host)."""
    off = np.empty(n + 1, dtype=np.uint64)
    check(_lib.load().icsw_mixed_offsets(off.ctypes.data, n, seed))
    return off


def as_u16(t):
    return t.cpu().numpy().view(np.uint16)


def as_u32(t):
    return t.cpu().numpy().view(np.uint32)
