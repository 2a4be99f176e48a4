"""GPU: the host-memory entry points on per-tick batch sizes (the TUN /
socket event loop's few datagrams per tick, util/tuntap/tuntap_adapter.cpp:5-21
inside util/tcp_minnow_socket/tcp_minnow_socket.h:138-164).

A host batch that fits one staging chunk and at most `zero_copy_max` bytes
is not DMA'd: the kernel reads the page-locked bytes (the caller's own when
they are page-locked, the staging slot's otherwise), offsets, inits and
messages over PCIe and writes its results into the page-locked result area
(icsum_host.cpp, DESIGN.md §6 "Per-tick host batches").  Every case runs on
three engines — the default threshold, zero-copy off (zero_copy_max=0: the
DMA path on the same sizes) and zero-copy for every one-chunk batch
(zero_copy_max=2^30) — against the oracle, from pageable and page-locked
memory, at odd starts, with the calls of different sizes and kinds
interleaved on one engine so a result area reused between calls cannot
pass on stale results."""
import numpy as np
import pytest

from conftest import force_id
from helpers import pack_contiguous

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["auto", "0", str(1 << 30)])
def zeng(request):
    from conftest import engine_with

    yield from engine_with(None if request.param == "auto" else {"zero_copy_max": request.param})


def _host(buf, pinned):
    import torch

    h = torch.empty(buf.size, dtype=torch.uint8, pin_memory=pinned).numpy()
    h[:] = buf
    return h


@pytest.mark.parametrize("pinned", [False, True])
def test_zc_checksum_fixed_and_offsets(zeng, orc, pinned):
    rng = np.random.default_rng(41)
    for n in (1, 2, 17, 300, 5000):
        L = 1500
        buf = _host(rng.integers(0, 256, n * L + 3, dtype=np.uint8), pinned)
        init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        got = zeng.checksum_batch_host(buf, n, stride=L, seg_len=L - 1, init=init)
        assert (got == orc.checksum_batch(buf, n, stride=L, seg_len=L - 1, init=init)).all(), n
        lens = rng.integers(0, 3000, n)
        segs = [rng.integers(0, 256, int(x), dtype=np.uint8).tobytes() for x in lens]
        b2, off = pack_contiguous(segs, 3)
        h2 = _host(b2, pinned)
        got = zeng.checksum_batch_host(h2, n, offsets=off)
        assert (got == orc.checksum_batch(b2, n, offsets=off)).all(), n


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("lead", [0, 3])
def test_zc_ipv4_every_mode(zeng, orc, pinned, lead):
    from test_gpu_parity import _random_datagrams

    rng = np.random.default_rng(7 + lead)
    for n in (1, 7, 300):
        segs = _random_datagrams(rng, n)
        buf, off = pack_contiguous(segs, lead)
        for mode in (0, 1, 2):
            h = _host(buf, pinned)
            ip, tcp, st = zeng.ipv4_tcp_batch_host(h, n, mode, offsets=off)
            hb = buf.copy()
            w = orc.ipv4_tcp_batch(hb, n, mode, offsets=off)
            assert (ip == w[0]).all() and (tcp == w[1]).all() and (st == w[2]).all(), (n, mode)
            assert (h == hb).all(), (n, mode)
    # fixed stride, MTU-sized: PATCH, then VERIFY over the patched bytes
    n, L = 64, 1500
    data = orc.fill_bytes(0x10710002, 0, n * L)
    h = _host(data, pinned)
    zeng.ipv4_tcp_batch_host(h, n, 2, stride=L, dgram_len=L)
    ip, tcp, st = zeng.ipv4_tcp_batch_host(h, n, 1, stride=L, dgram_len=L)
    w = orc.ipv4_tcp_batch(h.copy(), n, 1, stride=L, dgram_len=L)
    assert (st == w[2]).all() and (tcp == w[1]).all() and (ip == w[0]).all()


@pytest.mark.parametrize("pinned", [False, True])
def test_zc_wrap_in_place_and_headers_apart(zeng, orc, pinned):
    from test_gpu_wrap import _oracle_wire, _random_batch

    rng = np.random.default_rng(99)
    for n in (1, 33, 500):
        segs, m = _random_batch(rng, n)
        want = _oracle_wire(orc, segs, m)
        buf, off = pack_contiguous(segs, 1)
        h = _host(buf, pinned)
        zeng.tcp_wrap_batch_host(h, m, n, offsets=off)
        for i, w in enumerate(want):
            assert h[off[i]:off[i + 1]].tobytes() == w, (n, i)
        pays = [s[40:] for s in segs]
        pb, poff = pack_contiguous(pays, 2)
        hdrs = zeng.tcp_wrap_headers_host(_host(pb, pinned), m, n, offsets=poff)
        for i, w in enumerate(want):
            assert hdrs[40 * i:40 * i + 40].tobytes() == w[:40], (n, i)


def test_zc_interleaved_calls_no_stale_results(zeng, orc):
    """Calls of different kinds and sizes in turn on one engine (the result
    areas of the staging slots are reused): each one equals the oracle."""
    from test_gpu_parity import _random_datagrams

    rng = np.random.default_rng(5)
    for r in range(12):
        n = int(rng.integers(1, 40))
        if r % 3 == 0:
            buf = rng.integers(0, 256, n * 576, dtype=np.uint8)
            got = zeng.checksum_batch_host(buf, n, stride=576, seg_len=576)
            assert (got == orc.checksum_batch(buf, n, stride=576, seg_len=576)).all(), r
        else:
            segs = _random_datagrams(rng, n)
            buf, off = pack_contiguous(segs, r % 4)
            mode = r % 3
            ip, tcp, st = zeng.ipv4_tcp_batch_host(buf.copy(), n, mode, offsets=off)
            w = orc.ipv4_tcp_batch(buf.copy(), n, mode, offsets=off)
            assert (ip == w[0]).all() and (tcp == w[1]).all() and (st == w[2]).all(), r


def test_zc_path_taken_per_threshold(zeng, orc, request):
    """ics_dispatch_info's host counters show which path each engine took, so
    a zero-copy path that silently stopped running (equal results either way)
    fails here: a 6 KB batch is read in place unless zero_copy_max=0; a 3 MB
    batch (above the default 2 MiB) is DMA'd unless the threshold is 2^30."""
    param = request.node.callspec.params["zeng"]
    rng = np.random.default_rng(17)
    for n, zc_expected in ((4, param != "0"), (2048, param == str(1 << 30))):
        buf = rng.integers(0, 256, n * 1500, dtype=np.uint8)
        a = zeng.dispatch_info()
        got = zeng.checksum_batch_host(buf, n, stride=1500, seg_len=1500)
        b = zeng.dispatch_info()
        assert (got == orc.checksum_batch(buf, n, stride=1500, seg_len=1500)).all(), n
        zc = b["host_zero_copy"] - a["host_zero_copy"]
        dma = b["host_dma_chunks"] - a["host_dma_chunks"]
        assert (zc, dma) == ((1, 0) if zc_expected else (0, 1)), (param, n, zc, dma)


def test_zc_completion_over_many_blocks_and_two_pass_wrap(orc):
    """The completion word comes from the launch's last block (a block-count
    ticket, icsum_kernels.hip signal_done): zero-copy launches of hundreds of
    blocks, back to back on every slot (the ticket word must be back at 0
    after each), and the two-pass wrap, whose header pass completes the call."""
    from conftest import engine_with
    from test_gpu_wrap import _oracle_wire, _random_batch

    rng = np.random.default_rng(0xD0E)
    for eng in engine_with({"zero_copy_max": str(1 << 30), "wrap_passes": "2"}):
        for r in range(8):
            n = int(rng.integers(1, 20000))
            L = int(rng.choice([64, 576, 1500]))
            buf = rng.integers(0, 256, n * L, dtype=np.uint8)
            a = eng.dispatch_info()["host_zero_copy"]
            got = eng.checksum_batch_host(buf, n, stride=L, seg_len=L)
            assert eng.dispatch_info()["host_zero_copy"] == a + 1, r
            assert (got == orc.checksum_batch(buf, n, stride=L, seg_len=L)).all(), (r, n, L)
            ip, tcp, st = eng.ipv4_tcp_batch_host(buf, n, 1, stride=L, dgram_len=L)
            w = orc.ipv4_tcp_batch(buf.copy(), n, 1, stride=L, dgram_len=L)
            assert (ip == w[0]).all() and (tcp == w[1]).all() and (st == w[2]).all(), (r, n, L)
        for n in (1, 700, 9000):
            segs, m = _random_batch(rng, n)
            want = _oracle_wire(orc, segs, m)
            buf, off = pack_contiguous(segs, 1)
            eng.tcp_wrap_batch_host(buf, m, n, offsets=off)
            for i, w in enumerate(want):
                assert buf[off[i]:off[i + 1]].tobytes() == w, (n, i)
            pb, poff = pack_contiguous([s[40:] for s in segs], 0)
            hdrs = eng.tcp_wrap_headers_host(pb, m, n, offsets=poff)
            for i, w in enumerate(want):
                assert hdrs[40 * i:40 * i + 40].tobytes() == w[:40], (n, i)


def test_zc_first_call_after_freed_device_memory(orc):
    """A context's first zero-copy call right after device memory full of
    0xFF bytes was freed (the C-ABI example's order: ics_malloc / ics_free,
    then a host call): the completion tickets the call allocates may reuse
    that memory, and the slots' non-blocking streams do not wait for the
    null stream's memset — ensure_staging zeroes the tickets on slot 0's
    stream and waits for that stream before any slot launches, so the ticket
    starts at 0 and the call completes (the round-4 c_abi_example failure,
    'completion word was not written')."""
    import ctypes

    from conftest import engine_with

    rng = np.random.default_rng(0x71C)
    for _ in range(3):
        for eng in engine_with({"zero_copy_max": str(1 << 30)}):
            ptrs = []
            junk = np.full(1 << 20, 0xFF, dtype=np.uint8)
            for _ in range(8):
                p = ctypes.c_void_p()
                assert eng.lib.ics_malloc(eng.ctx, ctypes.byref(p), junk.size) == 0
                assert eng.lib.ics_memcpy_htod(eng.ctx, p, junk.ctypes.data, junk.size, None) == 0
                ptrs.append(p)
            assert eng.lib.ics_stream_synchronize(eng.ctx, None) == 0
            for p in ptrs:
                assert eng.lib.ics_free(eng.ctx, p) == 0
            n, L = 64, 1500
            buf = rng.integers(0, 256, n * L, dtype=np.uint8)
            want = buf.copy()
            w = orc.ipv4_tcp_batch(want, n, 2, stride=L, dgram_len=L)
            ip, tcp, st = eng.ipv4_tcp_batch_host(buf, n, 2, stride=L, dgram_len=L)
            assert (ip == w[0]).all() and (tcp == w[1]).all() and (st == w[2]).all()
            assert (buf == want).all()  # PATCH wrote what the oracle wrote
            assert eng.dispatch_info()["host_zero_copy"] >= 1


def test_poisoned_ticket_fails_once_then_recovers(orc):
    """A slot whose block-count ticket is non-zero when a zero-copy launch
    starts (ICSUM_FORCE poison_ticket: slot 0's ticket set to 2^30 once the
    staging exists) never has a block draw the last ticket, so the call's
    completion word stays unwritten: that call fails with ICS_ERR_HIP, and
    wait_flag zeroes the slot's ticket before returning — the next call on
    the same context and slot is exact, and so are the ones after it.  A
    one-block launch (up to 16 MTU datagrams) draws no ticket: it succeeds on
    the poisoned slot and leaves the poison for the first multi-block call."""
    from conftest import engine_with
    from tcpip_network_protocol_stack_amd._lib import IcsumError

    rng = np.random.default_rng(0x71D)
    n, L = 48, 1500
    buf = rng.integers(0, 256, n * L, dtype=np.uint8)
    init = rng.integers(0, 1 << 32, n, dtype=np.uint32)
    want = orc.checksum_batch(buf, n, stride=L, seg_len=L, init=init)
    for eng in engine_with({"zero_copy_max": str(1 << 30), "poison_ticket": str(1 << 30)}):
        # 8 datagrams: one block, no ticket drawn — exact, the poison stays
        got = eng.checksum_batch_host(buf[:8 * L], 8, stride=L, seg_len=L, init=init[:8])
        assert (got == want[:8]).all()
        with pytest.raises(IcsumError) as e:
            eng.checksum_batch_host(buf, n, stride=L, seg_len=L, init=init)
        assert "icsum error -2" in str(e.value) and "completion word was not written" in str(e.value)
        for _ in range(3):  # recovered: slot 0 counts from zero again
            got = eng.checksum_batch_host(buf, n, stride=L, seg_len=L, init=init)
            assert (got == want).all()
        assert eng.dispatch_info()["host_zero_copy"] == 5


@pytest.mark.parametrize("pinned", [False, True])
def test_error_after_chunks_in_flight_drains_slots(orc, pinned):
    """A fused-IPv4 host batch (datagrams never split into pieces) whose last
    datagram is larger than a staging slot fails with ICS_ERR_INVALID after
    several 1 MiB chunks were enqueued; the call drains every slot before it
    returns, so the caller's buffer can be freed at once, and the engine's
    next calls are exact."""
    import os

    import torch

    from conftest import engine_with
    from tcpip_network_protocol_stack_amd._lib import IcsumError

    os.environ["ICSUM_HOST_SLOT_MB"] = "1"
    try:
        gen = engine_with()
        eng = next(gen)
    finally:
        os.environ.pop("ICSUM_HOST_SLOT_MB")
    try:
        rng = np.random.default_rng(8)
        lens = [1500] * 4000 + [(1 << 20) + 8]
        off = np.zeros(len(lens) + 1, dtype=np.uint64)
        off[1:] = np.cumsum(lens)
        h = torch.empty(int(off[-1]), dtype=torch.uint8, pin_memory=pinned)
        h.numpy()[:] = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
        with pytest.raises(IcsumError, match="exceeds"):
            eng.ipv4_tcp_batch_host(h.numpy(), len(lens), 1, offsets=off)
        del h  # freed right after the error
        torch.cuda.synchronize()
        buf = rng.integers(0, 256, 4000 * 1500, dtype=np.uint8)
        ip, tcp, st = eng.ipv4_tcp_batch_host(buf, 4000, 1, stride=1500, dgram_len=1500)
        w = orc.ipv4_tcp_batch(buf.copy(), 4000, 1, stride=1500, dgram_len=1500)
        assert (ip == w[0]).all() and (tcp == w[1]).all() and (st == w[2]).all()
    finally:
        next(gen, None)


@pytest.fixture(scope="module", params=["auto", "0"], ids=["tick", "no_tick"])
def tick_eng(request):
    from conftest import engine_with

    yield from engine_with(None if request.param == "auto" else {"tick_inline": request.param})


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("base", [0, 1, 14])
def test_tick_offsets_in_kernel_arguments(tick_eng, orc, pinned, base):
    """A zero-copy tick of <= 16 offsets segments runs k_tick, its offsets in
    the kernel arguments (no dependent PCIe read of them): checksum with and
    without inits and the fused IPv4 kernel in every mode, 1..16 segments of
    every header shape and of up to 5000 bytes (more than one 16 x 8 pass),
    at an unaligned address; 17 segments take the grid launches.  With
    tick_inline=0 the same calls take the per-segment kernels.  Every result
    equals the oracle's."""
    import torch

    from test_gpu_parity import _random_datagrams

    rng = np.random.default_rng(0x71C + base + 7 * pinned)
    want_tick = not tick_eng.forced
    for n in (1, 2, 5, 16, 17):
        segs = _random_datagrams(rng, n)
        segs[0] = segs[0] + rng.integers(0, 256, 3500, dtype=np.uint8).tobytes()  # a long one
        buf, off = pack_contiguous(segs, int(rng.integers(0, 16)))
        alloc = torch.empty(buf.size + base, dtype=torch.uint8, pin_memory=pinned).numpy()
        h = alloc[base:]
        h[:] = buf
        init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        for ini in (init, None):
            got = tick_eng.checksum_batch_host(h, n, offsets=off, init=ini)
            assert (got == orc.checksum_batch(buf, n, offsets=off, init=ini)).all(), (n, base)
            assert (tick_eng.dispatch_info()["kernel"] == "tick") == (want_tick and n <= 16), n
        for mode in (0, 1, 2):
            h[:] = buf
            hb = buf.copy()
            w = orc.ipv4_tcp_batch(hb, n, mode, offsets=off)
            ip, tcp, st = tick_eng.ipv4_tcp_batch_host(h, n, mode, offsets=off)
            assert (ip == w[0]).all() and (tcp == w[1]).all() and (st == w[2]).all(), (n, mode, base)
            assert (h == hb).all(), (n, mode, base)
            assert (tick_eng.dispatch_info()["kernel"] == "tick") == (want_tick and n <= 16), (n, mode)


# resident; leaves after 3 ms without a call; srv_pollers 4: every wave
# polls; srv_blocks 4: four resident blocks, ticks of up to 64 segments
SRV_FORCE = [{"tick_server": 3000, "srv_blocks": 1}, {"tick_server": 3000, "srv_blocks": 1, "srv_pollers": 4},
             {"tick_server": 3000, "srv_blocks": 4}, {"tick_server": 3000, "srv_blocks": 8},
             # descriptors and the tick's bytes in device memory the host writes through the BAR
             {"tick_server": 3000, "srv_blocks": 4, "srv_vram": 1}, {"tick_server": 3000, "srv_blocks": 1, "srv_vram": 1}]


@pytest.fixture(scope="module", params=SRV_FORCE, ids=force_id)
def srv_eng(request):
    from conftest import engine_with

    for eng in engine_with(request.param):
        eng.srv_max = 16 * request.param.get("srv_blocks", 1)  # the largest served tick
        yield eng
        eng.set_tick_server(0)


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("base", [0, 3])
def test_tick_server_vs_oracle(srv_eng, orc, pinned, base):
    """The resident tick server (ics_set_tick_server) takes every zero-copy
    call of <= 16 segments (<= 64 over four blocks, split into parts of 16)
    — checksum with and without inits, the fused IPv4 kernel in every mode,
    offsets and fixed strides, every header shape, a 3.5 KB segment,
    unaligned addresses — from its mailboxes, no launch; one segment more
    takes the launches.  Every result equals the oracle's."""
    import torch

    from test_gpu_parity import _random_datagrams

    rng = np.random.default_rng(0x5E7 + base + 5 * pinned)
    for n in (1, 2, 16, 17, 3, 33, 47, 64, 65, 100, 128, 129):
        if n > srv_eng.srv_max + 1:
            continue
        segs = _random_datagrams(rng, n)
        segs[0] = segs[0] + rng.integers(0, 256, 3500, dtype=np.uint8).tobytes()
        buf, off = pack_contiguous(segs, int(rng.integers(0, 16)))
        alloc = torch.empty(buf.size + base, dtype=torch.uint8, pin_memory=pinned).numpy()
        h = alloc[base:]
        h[:] = buf
        init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        want_kernel = "tick_server" if n <= srv_eng.srv_max else None
        for ini in (init, None):
            got = srv_eng.checksum_batch_host(h, n, offsets=off, init=ini)
            assert (got == orc.checksum_batch(buf, n, offsets=off, init=ini)).all(), (n, base)
            k = srv_eng.dispatch_info()["kernel"]
            assert (k == "tick_server") == (want_kernel is not None), (n, k)
        for mode in (0, 1, 2):
            h[:] = buf
            hb = buf.copy()
            w = orc.ipv4_tcp_batch(hb, n, mode, offsets=off)
            ip, tcp, st = srv_eng.ipv4_tcp_batch_host(h, n, mode, offsets=off)
            assert (ip == w[0]).all() and (tcp == w[1]).all() and (st == w[2]).all(), (n, mode, base)
            assert (h == hb).all(), (n, mode, base)
        # fixed stride (1500 B datagrams)
        L = 1500
        fb = np.zeros(n * L, dtype=np.uint8)
        for i, sg in enumerate(segs):
            fb[i * L:(i + 1) * L] = np.frombuffer((bytes(sg) + bytes(L))[:L], dtype=np.uint8)
        fa = torch.empty(fb.size + base, dtype=torch.uint8, pin_memory=pinned).numpy()
        fh = fa[base:]
        for mode in (1, 2):
            fh[:] = fb
            hb = fb.copy()
            w = orc.ipv4_tcp_batch(hb, n, mode, stride=L, dgram_len=L)
            ip, tcp, st = srv_eng.ipv4_tcp_batch_host(fh, n, mode, stride=L, dgram_len=L)
            assert (ip == w[0]).all() and (tcp == w[1]).all() and (st == w[2]).all(), (n, mode, base, "fixed")
            assert (fh == hb).all(), (n, mode, base, "fixed")


@pytest.mark.parametrize("blocks,vram", [(1, 0), (4, 0), (8, 0), (4, 1)])
def test_tick_server_idle_exit_relaunch_and_stop(orc, blocks, vram):
    """The server leaves after its idle time and the next call launches it
    again (exact results across many exits; with four blocks the grid
    leaves as a whole and ticks of 1..64 segments alternate); ics_set_tick_server(0) stops it
    (calls take k_tick), turning it back on resumes the server path, and
    ics_destroy with a resident server returns."""
    import time

    from conftest import engine_with

    rng = np.random.default_rng(0x5E8)
    segs = [rng.integers(0, 256, int(x), dtype=np.uint8).tobytes() for x in (40, 1500, 576, 1)]
    buf, off = pack_contiguous(segs, 5)
    want = orc.checksum_batch(buf, len(segs), offsets=off)
    big = [rng.integers(0, 256, int(x), dtype=np.uint8).tobytes() for x in rng.integers(0, 1500, 16 * blocks)]
    bbuf, boff = pack_contiguous(big, 7)
    bwant = orc.checksum_batch(bbuf, len(big), offsets=boff)
    for eng in engine_with({"tick_server": 500, "srv_blocks": blocks, "srv_vram": vram}):  # 0.5 ms idle: leaves between most calls
        for i in range(40):
            got = eng.checksum_batch_host(buf, len(segs), offsets=off)
            assert (got == want).all(), i
            assert eng.dispatch_info()["kernel"] == "tick_server"
            if i % 3 == 0:
                assert (eng.checksum_batch_host(bbuf, len(big), offsets=boff) == bwant).all(), i
                assert eng.dispatch_info()["kernel"] == "tick_server"
            time.sleep(0.002 if i % 2 else 0.0)
        eng.set_tick_server(0)
        assert (eng.checksum_batch_host(buf, len(segs), offsets=off) == want).all()
        assert eng.dispatch_info()["kernel"] == "tick"
        eng.set_tick_server(100000)
        for _ in range(5):
            assert (eng.checksum_batch_host(buf, len(segs), offsets=off) == want).all()
            assert eng.dispatch_info()["kernel"] == "tick_server"
        # leave it resident: the engine's close (ics_destroy) stops it


def test_tick_server_blocks_api(orc):
    """ics_set_tick_server_blocks: 1..8 accepted, 0 and 9 rejected with
    ICS_ERR_INVALID; the default is 4 (64 segments served, 65 launched);
    a change restarts the server and moves the served limit (2 blocks: 32
    served, 33 launched) — results equal to the oracle's either way."""
    from conftest import engine_with

    from tcpip_network_protocol_stack_amd._lib import IcsumError

    rng = np.random.default_rng(0x5EB)
    segs = [rng.integers(0, 256, int(x), dtype=np.uint8).tobytes() for x in rng.integers(1, 1500, 65)]
    for eng in engine_with({"tick_server": 20000}):
        for bad in (0, 9):
            with pytest.raises(IcsumError, match="blocks"):
                eng.set_tick_server_blocks(bad)
        for blocks, cases in ((None, (64, 65, 1)), (2, (32, 33, 16)), (8, (65, 17)), (1, (16, 17))):
            if blocks:
                eng.set_tick_server_blocks(blocks)
            limit = 16 * (blocks or 4)
            for n in cases:
                buf, off = pack_contiguous(segs[:n], 2)
                got = eng.checksum_batch_host(buf, n, offsets=off)
                assert (got == orc.checksum_batch(buf, n, offsets=off)).all(), (blocks, n)
                assert (eng.dispatch_info()["kernel"] == "tick_server") == (n <= limit), (blocks, n)
        eng.set_tick_server(0)


@pytest.mark.parametrize("pinned", [False, True])
def test_tick_server_wrap_vs_oracle(srv_eng, orc, pinned):
    """Wrap ticks on the server: ics_tcp_wrap_batch_host (headers written into
    the datagrams) and ics_tcp_wrap_headers_host (payloads alone, headers to
    an array) for 1..16 messages of 0..1460-byte payloads, offsets and fixed
    stride, against the oracle's serialize(wrap_tcp_in_ip(msg)); 17 take the
    launches (with four blocks: up to 64, 65 take the launches)."""
    import torch

    from test_gpu_wrap import _oracle_wire, _random_batch

    rng = np.random.default_rng(0x5E9 + pinned)
    for n in (1, 5, 16, 17, 40, 64, 65, 128, 129):
        if n > srv_eng.srv_max + 1:
            continue
        segs, m = _random_batch(rng, n)
        want = _oracle_wire(orc, segs, m)
        buf, off = pack_contiguous(segs, 3)
        h = torch.empty(buf.size, dtype=torch.uint8, pin_memory=pinned).numpy()
        h[:] = buf
        srv_eng.tcp_wrap_batch_host(h, m, n, offsets=off)
        assert (srv_eng.dispatch_info()["kernel"] == "tick_server") == (n <= srv_eng.srv_max), n
        for i, w in enumerate(want):
            assert h[off[i]:off[i + 1]].tobytes() == w, (n, i)
        pays = [s[40:] for s in segs]
        pb, poff = pack_contiguous(pays, 1)
        ph = torch.empty(pb.size, dtype=torch.uint8, pin_memory=pinned).numpy()
        ph[:] = pb
        hd = srv_eng.tcp_wrap_headers_host(ph, m, n, offsets=poff)
        for i, w in enumerate(want):
            assert hd[40 * i:40 * i + 40].tobytes() == w[:40], (n, i)
        # fixed stride: 1040-byte datagrams
        L = 1040
        _, m2 = _random_batch(rng, n, fixed=L - 40)
        body = rng.integers(0, 256, n * L, dtype=np.uint8)
        fh = torch.empty(body.size, dtype=torch.uint8, pin_memory=pinned).numpy()
        fh[:] = body
        srv_eng.tcp_wrap_batch_host(fh, m2, n, stride=L, dgram_len=L)
        for i in range(n):
            w = _oracle_wire(orc, [b"\0" * 40 + body[i * L + 40:(i + 1) * L].tobytes()], m2[i:i + 1])[0]
            assert fh[i * L:(i + 1) * L].tobytes() == w, (n, i, "fixed")


def test_tick_server_threads_and_two_contexts(orc):
    """Three threads call one engine's served host entry points at once (the
    context serialises its host calls: ics_ctx::mu) while a fourth drives a
    second engine whose own server is resident beside the first; checksum
    ticks with inits and VERIFY ticks of 1..16 segments from pageable and
    page-locked memory, every result equal to the oracle's."""
    from concurrent.futures import ThreadPoolExecutor

    import torch

    from conftest import engine_with
    from test_gpu_parity import _random_datagrams

    rng = np.random.default_rng(0x5EA)
    jobs = []
    for t in range(4):
        mine = []
        for k in range(24):
            n = int(rng.integers(1, 17))
            buf, off = pack_contiguous(_random_datagrams(rng, n), int(rng.integers(0, 16)))
            h = torch.empty(buf.size, dtype=torch.uint8, pin_memory=bool(k % 2)).numpy()
            h[:] = buf
            init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
            w = orc.ipv4_tcp_batch(buf.copy(), n, 1, offsets=off)
            mine.append((h, n, off, init, orc.checksum_batch(buf, n, offsets=off, init=init), w))
        jobs.append(mine)
    for e1 in engine_with({"tick_server": 20000}):
        for e2 in engine_with({"tick_server": 20000}):
            def run(t):
                eng = e1 if t < 3 else e2
                for rep in range(3):
                    for h, n, off, init, want_ck, w in jobs[t]:
                        assert (eng.checksum_batch_host(h, n, offsets=off, init=init) == want_ck).all(), (t, rep, n)
                        ip, tcp, st = eng.ipv4_tcp_batch_host(h, n, 1, offsets=off)
                        assert (ip == w[0]).all() and (tcp == w[1]).all() and (st == w[2]).all(), (t, rep, n)
                return True

            with ThreadPoolExecutor(4) as ex:
                assert all(ex.map(run, range(4)))
            assert e1.dispatch_info()["kernel"] == "tick_server"
            assert e2.dispatch_info()["kernel"] == "tick_server"
            e2.set_tick_server(0)
        e1.set_tick_server(0)


@pytest.mark.parametrize("force", [None, {"tick_server": 3000}], ids=["launched", "server"])
def test_host_offsets_not_monotone_rejected(orc, force):
    """A host batch whose offsets decrease anywhere — the first pair, inside
    a per-tick batch (k_tick / the tick server), inside a DMA'd batch — is
    ICS_ERR_INVALID ("not monotone") before any kernel reads it (a
    decreasing pair would otherwise reach a kernel as a segment of ~2^64
    bytes), for the checksum, fused IPv4 and wrap entries; the engine's next
    calls are exact."""
    from conftest import engine_with
    from tcpip_network_protocol_stack_amd._lib import IcsumError
    from test_gpu_parity import _random_datagrams
    from test_gpu_wrap import _random_batch

    rng = np.random.default_rng(0x0FF)
    for eng in engine_with(force):
        for n, bad in ((5, 0), (5, 2), (16, 15), (4000, 3000)):
            segs = _random_datagrams(rng, n)
            buf, off = pack_contiguous(segs, 3)
            wsegs, m = _random_batch(rng, n)
            wbuf, woff = pack_contiguous(wsegs, 1)
            for o in (off, woff):
                o[bad + 1] = o[bad] - 1  # offsets[bad] > offsets[bad + 1]
            with pytest.raises(IcsumError, match="not monotone"):
                eng.checksum_batch_host(buf, n, offsets=off)
            with pytest.raises(IcsumError, match="not monotone"):
                eng.ipv4_tcp_batch_host(buf, n, 1, offsets=off)
            with pytest.raises(IcsumError, match="not monotone"):
                eng.tcp_wrap_batch_host(wbuf, m, n, offsets=woff)
            # and the engine goes on exactly
            good, goff = pack_contiguous(segs, 3)
            assert (eng.checksum_batch_host(good, n, offsets=goff) == orc.checksum_batch(good, n, offsets=goff)).all()
