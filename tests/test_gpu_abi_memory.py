"""GPU: the C-ABI's memory helpers (include/icsum.h "memory" block) through
the raw entry points, the way a caller binding only the C header uses them
(INTEGRATION.md §2): ics_malloc / ics_memcpy_htod / ics_memcpy_dtoh /
ics_free, ics_host_alloc / ics_host_free, ics_device_of and
ics_stream_synchronize.  A round trip through device memory and through
page-locked memory is byte-exact, a batch in ics_host_alloc memory goes
through ics_checksum_batch_host (DMA'd without a staging copy) with the
oracle's results, and null outputs are ICS_ERR_INVALID, not a crash."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ICS_ERR_INVALID = -1


def test_memory_entry_points(orc):
    from conftest import engine_with

    rng = np.random.default_rng(0xAB1)
    for eng in engine_with():
        lib, ctx = eng.lib, eng.ctx
        dev = ctypes.c_int(-1)
        assert lib.ics_device_of(ctx, ctypes.byref(dev)) == 0 and dev.value == 0
        assert lib.ics_device_of(ctx, None) == ICS_ERR_INVALID
        assert lib.ics_malloc(ctx, None, 16) == ICS_ERR_INVALID
        assert lib.ics_host_alloc(ctx, None, 16) == ICS_ERR_INVALID
        for nbytes in (1, 4097, 1 << 20):
            src = rng.integers(0, 256, nbytes, dtype=np.uint8)
            back = np.zeros(nbytes, dtype=np.uint8)
            d, h = ctypes.c_void_p(), ctypes.c_void_p()
            assert lib.ics_malloc(ctx, ctypes.byref(d), nbytes) == 0 and d.value
            assert lib.ics_host_alloc(ctx, ctypes.byref(h), nbytes) == 0 and h.value
            pinned = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(h.value))
            assert lib.ics_memcpy_htod(ctx, d, src.ctypes.data, nbytes, None) == 0
            assert lib.ics_memcpy_dtoh(ctx, h, d, nbytes, None) == 0
            assert lib.ics_stream_synchronize(ctx, None) == 0
            assert np.array_equal(pinned, src), nbytes
            assert lib.ics_memcpy_dtoh(ctx, back.ctypes.data, d, nbytes, None) == 0
            assert lib.ics_stream_synchronize(ctx, None) == 0
            assert np.array_equal(back, src), nbytes
            # the page-locked copy as a host batch: 1500-byte segments (the last one short)
            n = (nbytes + 1499) // 1500
            off = np.minimum(np.arange(n + 1, dtype=np.uint64) * 1500, nbytes).astype(np.uint64)
            got = eng.checksum_batch_host(pinned, n, offsets=off)
            assert np.array_equal(got, orc.checksum_batch(src, n, offsets=off)), nbytes
            del pinned
            assert lib.ics_host_free(ctx, h) == 0
            assert lib.ics_free(ctx, d) == 0
        # zero-byte requests allocate and free like any other; null frees are no-ops
        d = ctypes.c_void_p()
        assert lib.ics_malloc(ctx, ctypes.byref(d), 0) == 0 and d.value
        assert lib.ics_free(ctx, d) == 0 and lib.ics_free(ctx, None) == 0 and lib.ics_host_free(ctx, None) == 0
        assert lib.ics_memcpy_htod(ctx, None, None, 0, None) == 0
