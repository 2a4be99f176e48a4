"""TEST INFRASTRUCTURE ONLY — ctypes view of the CPU oracle (oracle/_build/liboracle.so)
and of the real reference's InternetChecksum (oracle/_ref/libref_icsum.so, when built).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only to CHECK or to TIME a CPU baseline — never as the product.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "_build", "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_icsum.so")

_p, _u64, _int = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int


class _Cksum(ctypes.Structure):
    _fields_ = [("sum", ctypes.c_uint32), ("parity", ctypes.c_int)]


_SIG = {
    "orc_init": (None, [ctypes.POINTER(_Cksum), ctypes.c_uint32]),
    "orc_add": (None, [ctypes.POINTER(_Cksum), _p, ctypes.c_size_t]),
    "orc_value": (ctypes.c_uint16, [ctypes.POINTER(_Cksum)]),
    "orc_fold": (ctypes.c_uint16, [ctypes.c_uint32]),
    "orc_checksum_batch": (None, [_p, _p, _u64, _u64, _p, _p, _u64]),
    "orc_sum_batch": (None, [_p, _p, _u64, _u64, _p, _p, _p, _u64]),
    "orc_checksum_batch_mt": (_int, [_p, _p, _u64, _u64, _p, _p, _u64, _int]),
    "orc_ipv4_tcp": (None, [_p, _u64, _int, ctypes.POINTER(ctypes.c_uint16),
                            ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(ctypes.c_uint8)]),
    "orc_ipv4_tcp_batch": (None, [_p, _p, _u64, _u64, _u64, _int, _p, _p, _p]),
    "orc_router_ttl": (None, [_p, _u64, ctypes.POINTER(ctypes.c_uint8)]),
    "orc_sm64": (_u64, [_u64]),
    "orc_word": (_u64, [_u64, _u64]),
    "orc_fill_bytes": (None, [_u64, _u64, _u64, _p]),
    "orc_pseudo_init": (ctypes.c_uint32, [_u64, _u64, _u64]),
    "orc_mixed_len": (_u64, [_u64, _u64]),
    "orc_ipv4_tcp_headers": (None, [_u64, _u64, _u64, _p]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-s", "-C", HERE])
        l = ctypes.CDLL(ORACLE_SO)
        for k, (r, a) in _SIG.items():
            f = getattr(l, k)
            f.restype = r
            f.argtypes = a
        _lib = l
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


def _buf(b):
    if isinstance(b, (bytes, bytearray)):
        return np.frombuffer(bytes(b), dtype=np.uint8)
    return np.ascontiguousarray(b, dtype=np.uint8)


class InternetChecksum:
    """Restatement of util/tools/checksum.h:9-60 with the same method names."""

    def __init__(self, init=0):
        self._c = _Cksum()
        lib().orc_init(ctypes.byref(self._c), init & 0xFFFFFFFF)

    def add(self, data):
        if isinstance(data, (list, tuple)):
            for piece in data:
                self.add(piece)
            return
        a = _buf(data)
        lib().orc_add(ctypes.byref(self._c), _ptr(a), a.size)

    def value(self):
        return lib().orc_value(ctypes.byref(self._c))

    @property
    def sum(self):
        return self._c.sum


def fold(s):
    return lib().orc_fold(s & 0xFFFFFFFF)


def checksum_batch(data, n, offsets=None, stride=0, seg_len=0, init=None, threads=1):
    data = _buf(data)
    out = np.empty(n, dtype=np.uint16)
    off = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    ini = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
    if threads > 1:
        lib().orc_checksum_batch_mt(_ptr(data), _ptr(off), stride, seg_len, _ptr(ini), _ptr(out), n, threads)
    else:
        lib().orc_checksum_batch(_ptr(data), _ptr(off), stride, seg_len, _ptr(ini), _ptr(out), n)
    return out


def sum_batch(data, n, offsets=None, stride=0, seg_len=0, init=None, odd=None):
    data = _buf(data)
    out = np.empty(n, dtype=np.uint32)
    off = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    ini = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
    od = None if odd is None else np.ascontiguousarray(odd, dtype=np.uint8)
    lib().orc_sum_batch(_ptr(data), _ptr(off), stride, seg_len, _ptr(ini), _ptr(od), _ptr(out), n)
    return out


def ipv4_tcp(dgram, mode):
    """One raw datagram -> (ip_ck, tcp_ck, status, bytes-after-patch)."""
    a = bytearray(dgram)
    buf = (ctypes.c_uint8 * max(len(a), 1)).from_buffer(a) if a else (ctypes.c_uint8 * 1)()
    ip, tcp, st = ctypes.c_uint16(), ctypes.c_uint16(), ctypes.c_uint8()
    lib().orc_ipv4_tcp(ctypes.addressof(buf), len(a), mode, ctypes.byref(ip), ctypes.byref(tcp), ctypes.byref(st))
    return ip.value, tcp.value, st.value, bytes(a)


def ipv4_tcp_batch(dgrams, n, mode, offsets=None, stride=0, dgram_len=0):
    """dgrams: writable uint8 numpy array (patched in place in PATCH mode)."""
    ip = np.empty(n, dtype=np.uint16)
    tcp = np.empty(n, dtype=np.uint16)
    st = np.empty(n, dtype=np.uint8)
    off = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    lib().orc_ipv4_tcp_batch(_ptr(dgrams), _ptr(off), stride, dgram_len, n, mode, _ptr(ip), _ptr(tcp), _ptr(st))
    return ip, tcp, st


def router_ttl(dgram):
    a = bytearray(dgram)
    buf = (ctypes.c_uint8 * max(len(a), 1)).from_buffer(a) if a else (ctypes.c_uint8 * 1)()
    st = ctypes.c_uint8()
    lib().orc_router_ttl(ctypes.addressof(buf), len(a), ctypes.byref(st))
    return st.value, bytes(a)


# ---- workload spec --------------------------------------------------------
def fill_bytes(seed, pos0, n):
    out = np.empty(n, dtype=np.uint8)
    lib().orc_fill_bytes(seed, pos0, n, _ptr(out))
    return out


def pseudo_init(seed, i, length):
    return lib().orc_pseudo_init(seed, i, length)


def pseudo_inits(seed, n, length=None, offsets=None, index0=0):
    out = np.empty(n, dtype=np.uint32)
    for i in range(n):
        L = int(offsets[i + 1] - offsets[i]) if offsets is not None else length
        out[i] = lib().orc_pseudo_init(seed, index0 + i, L)
    return out


def mixed_len(seed, i):
    return lib().orc_mixed_len(seed, i)


def ipv4_tcp_headers(seed, i, dgram_len, buf):
    """Overwrite header fields of one datagram in `buf` (writable uint8 array)."""
    lib().orc_ipv4_tcp_headers(seed, i, dgram_len, _ptr(buf))


# ---- the real reference (CPU baseline, kind "reference") -------------------
_ref = None


def ref_lib():
    """oracle/_ref/libref_icsum.so (reference InternetChecksum) or None."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        l = ctypes.CDLL(REF_SO)
        l.ref_checksum_batch.restype = _int
        l.ref_checksum_batch.argtypes = [_p, _p, _u64, _u64, _p, _p, _u64, _int]
        _ref = l
    return _ref
