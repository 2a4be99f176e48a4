"""ctypes binding of libicsum.so (the C-ABI declared in include/icsum.h).

This is the same binding a maintainer would add to call the engine from any
FFI.  Loading fails loudly: there is no Python or CPU
fallback for the checksum path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libicsum.so")
# the same engine with every device load bounds-checked (slower,
# synchronises after each call; ICS_ERR_INVALID "bounds check: ..." on a fault)
DEBUG_LIB_PATH = os.path.join(_HERE, "libicsum_debug.so")

ICS_OK = 0
ICS_MODE_COMPUTE, ICS_MODE_VERIFY, ICS_MODE_PATCH = 0, 1, 2
ICS_ST_IPV4_OK, ICS_ST_TCP_CKSUM_OK, ICS_ST_TCP_HDR_OK, ICS_ST_PROTO_TCP = 0x01, 0x02, 0x04, 0x08
ICS_ST_ACCEPT = 0x0F
ICS_BINNING_AUTO, ICS_BINNING_SINGLE, ICS_BINNING_BINNED = -1, 0, 1
ICS_TCP_FIN, ICS_TCP_SYN, ICS_TCP_RST, ICS_TCP_ACK = 0x01, 0x02, 0x04, 0x10


class TcpMsg(ctypes.Structure):
    """struct ics_tcp_msg (include/icsum.h), 28 bytes: the fields
    wrap_tcp_in_ip puts on the wire (util/tcp_over_ip/tcp_over_ip.cpp:69-88)."""
    _fields_ = [("src", ctypes.c_uint32), ("dst", ctypes.c_uint32), ("seqno", ctypes.c_uint32),
                ("ackno", ctypes.c_uint32), ("src_port", ctypes.c_uint16), ("dst_port", ctypes.c_uint16),
                ("window", ctypes.c_uint16), ("flags", ctypes.c_uint8), ("ttl", ctypes.c_uint8),
                ("id", ctypes.c_uint16), ("reserved", ctypes.c_uint16)]


assert ctypes.sizeof(TcpMsg) == 28


class DispatchInfo(ctypes.Structure):
    """struct ics_dispatch_info_t (include/icsum.h): the last call's launch and
    the plan cache's counters."""
    _fields_ = [("plan_hits", ctypes.c_uint64), ("plan_misses", ctypes.c_uint64),
                ("plan_requests", ctypes.c_uint64), ("last_kernel", ctypes.c_int32),
                ("last_lps", ctypes.c_int32), ("last_unroll", ctypes.c_int32), ("last_plan", ctypes.c_int32),
                ("host_zero_copy", ctypes.c_uint64), ("host_dma_chunks", ctypes.c_uint64)]


class SegBatch(ctypes.Structure):
    """struct ics_seg_batch (include/icsum.h): one ics_checksum_batch call's arguments."""
    _fields_ = [("bytes", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("stride", ctypes.c_uint64),
                ("seg_len", ctypes.c_uint64), ("n", ctypes.c_uint64), ("init", ctypes.c_void_p),
                ("out", ctypes.c_void_p)]


class DgramBatch(ctypes.Structure):
    """struct ics_dgram_batch (include/icsum.h): one ics_ipv4_tcp_batch call's arguments."""
    _fields_ = [("dgrams", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("stride", ctypes.c_uint64),
                ("dgram_len", ctypes.c_uint64), ("n", ctypes.c_uint64), ("ip_ck", ctypes.c_void_p),
                ("tcp_ck", ctypes.c_void_p), ("status", ctypes.c_void_p)]


# ICS_K_* kernel ids of ics_dispatch_info_t.last_kernel
KERNELS = {1: "checksum", 2: "small", 3: "tiny", 4: "dense", 5: "twoclass", 6: "binned", 7: "ipv4",
           8: "ipv4_twoclass", 9: "wrap", 10: "wrap_2pass", 11: "router", 12: "batchv", 13: "tile",
           14: "router_hdrs", 15: "tick", 16: "tick_server"}

_p = ctypes.c_void_p
_u64 = ctypes.c_uint64
_int = ctypes.c_int

# name -> (restype, argtypes); every symbol include/icsum.h and
# include/icsum_workload.h declare
SIGNATURES = {
    "ics_version": (ctypes.c_char_p, []),
    "ics_abi_version": (_int, []),
    "ics_device_count": (_int, [ctypes.POINTER(_int)]),
    "ics_create": (_int, [_int, ctypes.POINTER(_p)]),
    "ics_destroy": (_int, [_p]),
    "ics_device_of": (_int, [_p, ctypes.POINTER(_int)]),
    "ics_last_error": (ctypes.c_char_p, []),
    "ics_checksum_batch": (_int, [_p, _p, _p, _u64, _u64, _p, _p, _u64, _p]),
    "ics_sum_batch": (_int, [_p, _p, _p, _u64, _u64, _p, _p, _p, _u64, _p]),
    "ics_set_binning": (_int, [_p, _int]),
    "ics_set_tick_server": (_int, [_p, ctypes.c_uint32]),
    "ics_set_tick_server_blocks": (_int, [_p, ctypes.c_uint32]),
    "ics_fold_batch": (_int, [_p, _p, _p, _u64, _p]),
    "ics_ipv4_tcp_batch": (_int, [_p, _p, _p, _u64, _u64, _u64, _int, _p, _p, _p, _p]),
    "ics_router_ttl_batch": (_int, [_p, _p, _p, _u64, _u64, _u64, _p, _p]),
    "ics_router_ttl_headers": (_int, [_p, _p, _p, _u64, _u64, _u64, _p, _p, _p]),
    "ics_tcp_wrap_batch": (_int, [_p, _p, _p, _u64, _u64, _u64, _p, _p, _p, _p]),
    "ics_tcp_wrap_batch_host": (_int, [_p, _p, _p, _u64, _u64, _u64, _p]),
    "ics_tcp_wrap_headers": (_int, [_p, _p, _p, _u64, _u64, _u64, _p, _p, _p, _p, _p]),
    "ics_tcp_wrap_headers_host": (_int, [_p, _p, _p, _u64, _u64, _u64, _p, _p]),
    "ics_checksum_batch_host": (_int, [_p, _p, _p, _u64, _u64, _p, _p, _u64]),
    "ics_ipv4_tcp_batch_host": (_int, [_p, _p, _p, _u64, _u64, _u64, _int, _p, _p, _p]),
    "ics_malloc": (_int, [_p, ctypes.POINTER(_p), ctypes.c_size_t]),
    "ics_free": (_int, [_p, _p]),
    "ics_host_alloc": (_int, [_p, ctypes.POINTER(_p), ctypes.c_size_t]),
    "ics_host_free": (_int, [_p, _p]),
    "ics_memcpy_htod": (_int, [_p, _p, _p, ctypes.c_size_t, _p]),
    "ics_memcpy_dtoh": (_int, [_p, _p, _p, ctypes.c_size_t, _p]),
    "ics_stream_synchronize": (_int, [_p, _p]),
    "ics_dispatch_info": (_int, [_p, ctypes.POINTER(DispatchInfo)]),
    "ics_checksum_batchv": (_int, [_p, ctypes.POINTER(SegBatch), ctypes.c_uint32, _p]),
    "ics_ipv4_tcp_batchv": (_int, [_p, ctypes.POINTER(DgramBatch), ctypes.c_uint32, _int, _p]),
    "icsw_fill_bytes": (_int, [_p, _p, _u64, _u64, _u64, _p]),
    "icsw_pseudo_inits": (_int, [_p, _p, _p, _u64, _u64, _u64, _u64, _p]),
    "icsw_ipv4_tcp_headers": (_int, [_p, _p, _u64, _u64, _u64, _u64, _u64, _p]),
    "icsw_mixed_len": (_u64, [_u64, _u64]),
    "icsw_mixed_offsets": (_int, [_p, _u64, _u64]),
}


class IcsumError(RuntimeError):
    pass


_libs = {}
_current = None  # the library check() reads ics_last_error() from


def load(path=None):
    """Load libicsum.so (or `path`, e.g. DEBUG_LIB_PATH), built by
    __graft_entry__.build(); raise if absent.  Each path is loaded once."""
    global _current
    path = path or LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise IcsumError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the checksum engine has no CPU fallback)")
    # torch (if imported) already holds the process's libamdhip64.so.7; the
    # engine binds to the same runtime by soname.
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _libs[path] = lib
    if path == LIB_PATH or _current is None:
        _current = lib
    return lib


def check(rc, lib=None):
    if rc != ICS_OK:
        msg = (lib or _current or load()).ics_last_error().decode(errors="replace")
        raise IcsumError(f"icsum error {rc}: {msg}")
    return rc
