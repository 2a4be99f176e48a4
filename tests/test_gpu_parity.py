"""GPU parity: the HIP path through the C-ABI (libicsum.so) against the golden
vectors of the real reference and against the oracle on seeded inputs.

Bar: bit-exact (integer / byte work).  Every call goes through libicsum.so;
torch only allocates device memory."""
import hashlib
import os

import numpy as np
import pytest

from conftest import engine_with, force_id, golden
from helpers import kat_cases, pack_contiguous, wires

pytestmark = pytest.mark.gpu

# every instantiated (LPS, UNROLL, MODE) of k_checksum the dispatch can reach —
# keep in sync with ICS_GEOMETRIES in icsum_kernels.hip (MODE 2: 16-byte grid
# fully masked, 3: 128-byte-line grid with primed boundary loads) — plus MODE
# 4, k_checksum_tiny (one lane per segment)
GEOMETRIES = [(4, 1, 2), (4, 2, 2), (8, 2, 2), (8, 8, 3), (16, 4, 3), (16, 5, 3), (16, 6, 3), (16, 7, 3), (16, 8, 3),
              (32, 8, 3), (64, 8, 3), (1, 4, 4)]
# small-segment kernel (k_checksum_small): (LPS, UNROLL, MODE unused, SEGS) — ICS_SMALL_GEOMETRIES
SMALL_GEOMETRIES = [(4, 1, 0, 2), (4, 2, 0, 2), (8, 2, 0, 2)]


_SIGNED = {np.dtype(np.uint16): np.int16, np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64}


def _t(a, dev="cuda:0"):
    """numpy -> device tensor; unsigned words travel as same-width signed views."""
    import torch

    a = np.ascontiguousarray(a)
    if a.dtype in _SIGNED:
        a = a.view(_SIGNED[a.dtype])
    if not a.flags.writeable:  # e.g. np.frombuffer over bytes: torch wants a writable array
        a = a.copy()
    return torch.from_numpy(a).to(dev)


def _u16(t):
    return t.cpu().numpy().view(np.uint16)


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module", params=GEOMETRIES + SMALL_GEOMETRIES,
                ids=lambda g: f"lps{g[0]}x{g[1]}m{g[2]}" + (f"s{g[3]}" if len(g) > 3 else ""))
def geo_engine(request):
    """An engine per lane-group geometry (forced through the ICSUM_FORCE hook)."""
    force = dict(zip(("lps", "unroll", "mode", "segs"), request.param))
    gen = _engine_with(force)
    eng = next(gen)
    eng.forced = request.param
    yield eng
    next(gen, None)


def _assert_forced(eng):
    """the forced geometry is the one that ran (an uninstantiated shape would
    silently fall back to the default and test nothing new)"""
    info = eng.dispatch_info()
    lps, unroll, mode = eng.forced[:3]
    kernel = "tiny" if mode == 4 else ("small" if len(eng.forced) > 3 else "checksum")
    assert (info["kernel"], info["lps"], info["unroll"]) == (kernel, lps, unroll), (info, eng.forced)


def _engine_with(force):
    yield from engine_with(force)


# length binning of offsets batches: forced split into bins (plan 1) or whole
# batch through the last bin's launch (plan 0), the on-device plan, tiny grids
# (many ticketed runs per block), and bin=0 (single-geometry dispatch)
BIN_ENVS = [{"bin": 1, "bin_plan": 1},
            {"bin": 1, "bin_plan": 1, "bin_blocks": 3},
            {"bin": 1, "bin_plan": 0, "bin_blocks": 5},
            # the 32-lane last-bin launch (auto above 1 M segments) under both plans
            {"bin": 1, "bin_plan": 0, "last_bin_lps": 32},
            {"bin": 1, "bin_plan": 1, "last_bin_lps": 32},
            # the whole batch in 16-lane groups from the last bin's launch
            {"bin": 1, "bin_plan": 2},
            {"bin": 1, "bin_plan": 2, "last_bin_lps": 32, "last_bin_blocks": 7},
            # ... or through the small-segment body
            {"bin": 1, "bin_plan": 3},
            {"bin": 1, "bin_plan": 3, "last_bin_lps": 32, "last_bin_blocks": 5},
            {"bin": 1},
            {"bin": 0}]


@pytest.fixture(scope="module", params=BIN_ENVS, ids=force_id)
def bin_engine(request):
    yield from _engine_with(request.param)


# ---------------------------------------------------------------- a1-a4 --
def test_kat_all_geometries(geo_engine):
    cases = kat_cases({"rfc1071", "len", "init", "whole"})
    segs = [b"".join(p) for _, p, _, _ in cases]
    want = [c[2] for c in cases]
    for lead in (0, 1, 6, 15):
        buf, off = pack_contiguous(segs, lead)
        init = np.array([c[0] for c in cases], dtype=np.uint32)
        out = geo_engine.checksum_batch(_t(buf), offsets=_t(off), init=_t(init))
        assert _u16(out).tolist() == want, f"lead={lead}"
        _assert_forced(geo_engine)


def test_kat_fill_and_wrap(engine):
    # long all-0x00 / all-0xFF segments incl. the uint32 wrap past 131074 bytes
    cases = kat_cases({"fill"})
    segs = [b"".join(p) for _, p, _, _ in cases]
    for lead in (0, 3):
        buf, off = pack_contiguous(segs, lead)
        init = np.array([c[0] for c in cases], dtype=np.uint32)
        out = engine.checksum_batch(_t(buf), offsets=_t(off), init=_t(init))
        assert _u16(out).tolist() == [c[2] for c in cases]


def test_split_pieces_chain(engine):
    # add(vector<string>) with parity carried across pieces (checksum.h:44-59):
    # chain ics_sum_batch piece by piece, then ics_fold_batch
    import torch

    cases = kat_cases({"split"})
    maxp = max(len(p) for _, p, _, _ in cases)
    sums = np.array([c[0] for c in cases], dtype=np.uint32)
    odd = np.zeros(len(cases), dtype=np.uint8)
    for k in range(maxp):
        segs = [p[k] if k < len(p) else b"" for _, p, _, _ in cases]
        buf, off = pack_contiguous(segs, 1)
        s = engine.sum_batch(_t(buf), offsets=_t(off), init=_t(sums), odd=_t(odd))
        sums = _u32(s).copy()
        odd ^= np.array([len(x) & 1 for x in segs], dtype=np.uint8)
    vals = engine.fold_batch(_t(sums))
    assert _u16(vals).tolist() == [c[2] for c in cases]
    torch.cuda.synchronize()


def test_random_differential(geo_engine, orc):
    rng = np.random.default_rng(20250225)
    n = 3000
    lens = rng.integers(0, 5000, n)
    lens[::97] = rng.integers(5000, 70000, lens[::97].size)  # some long ones
    lens[::113] = 0
    segs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
    buf, off = pack_contiguous(segs, 7)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    out = geo_engine.checksum_batch(_t(buf), offsets=_t(off), init=_t(init))
    want = orc.checksum_batch(buf, n, offsets=off, init=init)
    assert (_u16(out) == want).all()
    odd = rng.integers(0, 2, n).astype(np.uint8)
    sums = geo_engine.sum_batch(_t(buf), offsets=_t(off), init=_t(init), odd=_t(odd))
    assert (_u32(sums) == orc.sum_batch(buf, n, offsets=off, init=init, odd=odd)).all()


def _bin_lengths(rng, n):
    """Lengths over every bin (<= 144, <= 896, <= 1920, <= 4096, longer),
    zero-length segments and a few past the uint32 wrap of 0xFF bytes."""
    edges = [0, 1, 143, 144, 145, 895, 896, 897, 1919, 1920, 1921, 4095, 4096, 4097]
    lens = rng.choice([40, 64, 100, 576, 1500, 3000, 9000, 40000], n)
    lens = lens + rng.integers(-7, 8, n)
    lens[: len(edges)] = edges
    lens[len(edges)::101] = 0
    return lens.astype(np.int64)


def test_binned_differential(bin_engine, orc):
    rng = np.random.default_rng(0xB1)
    n = 6000
    segs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in _bin_lengths(rng, n)]
    for lead in (0, 5):
        buf, off = pack_contiguous(segs, lead)
        init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        out = bin_engine.checksum_batch(_t(buf), offsets=_t(off), init=_t(init))
        assert (_u16(out) == orc.checksum_batch(buf, n, offsets=off, init=init)).all(), f"lead={lead}"
        odd = rng.integers(0, 2, n).astype(np.uint8)
        sums = bin_engine.sum_batch(_t(buf), offsets=_t(off), init=_t(init), odd=_t(odd))
        assert (_u32(sums) == orc.sum_batch(buf, n, offsets=off, init=init, odd=odd)).all()
        out0 = bin_engine.checksum_batch(_t(buf), offsets=_t(off))  # init NULL = 0
        assert (_u16(out0) == orc.checksum_batch(buf, n, offsets=off)).all()


def test_binned_kats(bin_engine):
    # every KAT (incl. the 131076-byte 0xFF wrap) through the binned path
    cases = kat_cases({"rfc1071", "len", "init", "whole", "fill"})
    segs = [b"".join(p) for _, p, _, _ in cases]
    buf, off = pack_contiguous(segs, 3)
    init = np.array([c[0] for c in cases], dtype=np.uint32)
    out = bin_engine.checksum_batch(_t(buf), offsets=_t(off), init=_t(init))
    assert _u16(out).tolist() == [c[2] for c in cases]


def test_binned_bimodal_large(bin_engine, orc):
    # ACK-sized + MSS-sized segments interleaved (the mix a TCP receive path
    # sees), above the auto-binning threshold
    rng = np.random.default_rng(0xACC)
    n = 150_000
    lens = np.where(rng.random(n) < 0.5, 40, 1460) + rng.integers(0, 4, n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    off += 1
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    out = bin_engine.checksum_batch(_t(buf), offsets=_t(off))
    assert (_u16(out) == orc.checksum_batch(buf, n, offsets=off)).all()


def test_binned_ack_batch(bin_engine, orc):
    # ACK-sized segments (0-60 B, mean ~30 B): under the small-segment plan
    # the device runs one lane per segment (k_checksum_tiny's body inside the
    # last bin's launch), and on the second call the plan cache's single
    # launch does the same from the host; every dispatch gives the reference
    rng = np.random.default_rng(0xAC0)
    n = 70_000
    lens = rng.integers(0, 61, n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    off += 5
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = orc.checksum_batch(buf, n, offsets=off, init=init)
    d, doff, dinit = _t(buf), _t(off), _t(init)
    for call in range(3):
        assert (_u16(bin_engine.checksum_batch(d, offsets=doff, init=dinit)) == want).all(), call
    odd = rng.integers(0, 2, n).astype(np.uint8)
    sums = bin_engine.sum_batch(d, offsets=doff, init=dinit, odd=_t(odd))
    assert (_u32(sums) == orc.sum_batch(buf, n, offsets=off, init=init, odd=odd)).all()


def test_set_binning_modes(engine, orc):
    # ics_set_binning: every mode gives the same (reference) results; bad modes fail loudly
    from tcpip_network_protocol_stack_amd._lib import IcsumError

    rng = np.random.default_rng(0x5E7)
    n = 70_000  # above the AUTO threshold
    lens = rng.choice([20, 40, 576, 1460, 9000], n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    want = orc.checksum_batch(buf, n, offsets=off)
    try:
        for mode in (1, 0, -1):
            engine.set_binning(mode)
            assert (_u16(engine.checksum_batch(_t(buf), offsets=_t(off))) == want).all(), mode
        with pytest.raises(IcsumError):
            engine.set_binning(7)
    finally:
        engine.set_binning(-1)


def test_auto_plan_cache_repeated_and_changed_mix(engine, orc):
    """AUTO dispatch with the plan cache: the same long-segment batch (the
    device plans "whole batch") called repeatedly — the cached calls skip the
    binning passes and run that plan's single launch — then the SAME offsets
    buffer rewritten in place with a bimodal mix of the same n (a stale cache
    entry): every call's output equals the oracle's."""
    import torch

    rng = np.random.default_rng(0xCAC)
    n = 70_000
    lens = rng.integers(2048, 16384, n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    want = orc.checksum_batch(buf, n, offsets=off)
    dbuf, doff = _t(buf), _t(off)
    for k in range(40):
        out = engine.checksum_batch(dbuf, offsets=doff)
        if k % 7 == 0:
            torch.cuda.synchronize()
        assert (_u16(out) == want).all(), k
    lens2 = np.where(rng.random(n) < 0.5, 40, 1460)
    off2 = np.zeros(n + 1, dtype=np.uint64)
    off2[1:] = np.cumsum(lens2)
    doff.copy_(_t(off2))
    want2 = orc.checksum_batch(buf, n, offsets=off2)
    for k in range(70):  # past a re-plan (every 64th call) under the new mix
        assert (_u16(engine.checksum_batch(dbuf, offsets=doff)) == want2).all(), k


def _mix_lengths(rng, n, mix):
    """Segment lengths of the plan-cache tests' mixes: pure ACKs, MTU data,
    half and three quarters 40-byte ACKs among MTU segments (the 8-lane
    short-mix geometry), ACKs among jumbo segments (long bytes: not 8-lane)
    and long segments."""
    ack = lambda p, big: np.where(rng.random(n) < p, 40, big) + rng.integers(0, 4, n)  # noqa: E731
    return {"bimodal": lambda: ack(0.5, 1460), "ackheavy": lambda: ack(0.75, 1460),
            "ackjumbo": lambda: ack(0.75, 9000), "acks": lambda: rng.integers(40, 44, n),
            "mtu": lambda: rng.integers(1460, 1464, n), "long": lambda: rng.integers(4096, 9000, n)}[mix]()


@pytest.mark.parametrize("mix", ["acks", "mtu", "bimodal", "ackheavy", "ackjumbo", "long"])
def test_small_offsets_batch_plan_cache(engine, orc, mix):
    """Offsets batches below the binning threshold (16 Ki <= n < 64 Ki) take
    their single launch's geometry from the plan cached for the same offsets
    buffer (the plan kernels run behind the first and every 64th launch): 40
    repeated calls, then the same buffer rewritten with another mix; every
    output equals the oracle's."""
    import torch

    rng = np.random.default_rng(0x5A + len(mix))
    n = 20_000
    lens = _mix_lengths(rng, n, mix)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    lens2 = rng.integers(40, 9000, n)  # another mix, later, under the same pointer and n
    off2 = np.zeros(n + 1, dtype=np.uint64)
    off2[1:] = np.cumsum(lens2)
    buf = rng.integers(0, 256, int(max(off[-1], off2[-1])) + 16, dtype=np.uint8)  # holds both mixes
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = orc.checksum_batch(buf, n, offsets=off, init=init)
    dbuf, doff, dinit = _t(buf), _t(off), _t(init)
    for k in range(40):
        out = engine.checksum_batch(dbuf, offsets=doff, init=dinit)
        if k % 9 == 0:
            torch.cuda.synchronize()
        assert (_u16(out) == want).all(), (mix, k)
    doff.copy_(_t(off2))
    want2 = orc.checksum_batch(buf, n, offsets=off2, init=init)
    for k in range(20):
        assert (_u16(engine.checksum_batch(dbuf, offsets=doff, init=dinit)) == want2).all(), (mix, k)


@pytest.mark.parametrize("mix", ["bimodal", "ackheavy", "ackjumbo", "acks", "mtu", "long"])
def test_auto_plan_cache_every_whole_plan(engine, orc, mix):
    """Batches whose device plan is each of the whole-batch plans (whole,
    whole16, small body), the split plan and the 8-lane short mix, called 40
    times back to back: cached calls run the plan's single launch; then the
    same offsets buffer rewritten with the bimodal (or, for it, the long) mix
    and called 20 times more; every output equals the oracle's."""
    import torch

    rng = np.random.default_rng(len(mix))
    n = 300_000
    lens = _mix_lengths(rng, n, mix)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    off += 5
    off2 = np.zeros(n + 1, dtype=np.uint64)
    off2[1:] = np.cumsum(_mix_lengths(rng, n, "long" if mix == "bimodal" else "bimodal"))
    buf = rng.integers(0, 256, int(max(off[-1], off2[-1])) + 16, dtype=np.uint8)  # holds both mixes
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = orc.checksum_batch(buf, n, offsets=off, init=init)
    dbuf, doff, dinit = _t(buf), _t(off), _t(init)
    outs = [engine.checksum_batch(dbuf, offsets=doff, init=dinit) for _ in range(40)]
    for k, o in enumerate(outs):
        assert (_u16(o) == want).all(), k
    torch.cuda.synchronize()
    doff.copy_(_t(off2))
    want2 = orc.checksum_batch(buf, n, offsets=off2, init=init)
    outs = [engine.checksum_batch(dbuf, offsets=doff, init=dinit) for _ in range(70)]  # past a re-plan
    for k, o in enumerate(outs):
        assert (_u16(o) == want2).all(), (mix, k)


@pytest.mark.parametrize("stride,seg_len", [(1500, 1500), (1501, 1497), (64, 64), (9000, 9000),
                                            (16, 0), (24, 1), (9216, 9000), (7, 7)])
def test_fixed_stride(engine, orc, stride, seg_len):
    rng = np.random.default_rng(stride * 31 + seg_len)
    n = 2048 + 5
    buf = rng.integers(0, 256, n * stride + seg_len + 16, dtype=np.uint8)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    out = engine.checksum_batch(_t(buf), n=n, stride=stride, seg_len=seg_len, init=_t(init))
    assert (_u16(out) == orc.checksum_batch(buf, n, stride=stride, seg_len=seg_len, init=init)).all()
    out0 = engine.checksum_batch(_t(buf), n=n, stride=stride, seg_len=seg_len)  # init NULL = 0
    assert (_u16(out0) == orc.checksum_batch(buf, n, stride=stride, seg_len=seg_len)).all()


def test_empty_batch_and_single(engine, orc):
    import torch

    out = torch.full((4,), 7, dtype=torch.int16, device="cuda:0")
    engine.checksum_batch(_t(np.zeros(16, np.uint8)), n=0, stride=16, seg_len=16, out=out)
    assert _u16(out).tolist() == [7] * 4
    one = engine.checksum_batch(_t(np.frombuffer(bytes.fromhex("0001f203f4f5f6f7") + bytes(8), np.uint8)),
                                n=1, stride=8, seg_len=8)
    assert _u16(one).tolist() == [0x220D]


# ----------------------------------------------------- fused IPv4 + TCP ---
def _pack_wires(ws, lead=5):
    return pack_contiguous([bytes.fromhex(w) for w in ws], lead)


@pytest.mark.parametrize("lead", [0, 1, 2, 3])
def test_ipv4_tcp_verify_fixture(geo_engine, lead):
    cases = wires("tcp_wrap.json")
    buf, off = _pack_wires([c["wire"] for c in cases], lead)
    ip, tcp, st = geo_engine.ipv4_tcp_batch(_t(buf), 1, offsets=_t(off))
    ip, tcp, st = _u16(ip), _u16(tcp), st.cpu().numpy()
    for i, c in enumerate(cases):
        assert bool(st[i] & 1) == c["ip_parse_ok"], (i, c["tag"])
        if "tcp_parse_ok" in c:
            assert (st[i] & 6 == 6) == c["tcp_parse_ok"], (i, c["tag"])
            assert tcp[i] == c["tcp_value"] and ip[i] == c["ip_computed"], (i, c["tag"])
            assert bool(st[i] & 8) == (c["proto"] == 6)
        if c["tag"] == "wrap":
            assert st[i] == 0x0F


def test_ipv4_tcp_compute_and_patch_fixture(geo_engine):
    cases = wires("tcp_wrap.json", {"wrap"})
    good = [bytearray.fromhex(c["wire"]) for c in cases]
    junk = []
    for w in good:
        j = bytearray(w)
        j[10:12] = b"\x5a\xa5"
        j[36:38] = b"\xc3\x3c"
        junk.append(bytes(j))
    buf, off = pack_contiguous(junk, 3)
    d = _t(buf)
    ip, tcp, st = geo_engine.ipv4_tcp_batch(d, 0, offsets=_t(off))
    assert _u16(ip).tolist() == [c["ip_cksum"] for c in cases]
    assert _u16(tcp).tolist() == [w[36] << 8 | w[37] for w in good]
    assert (st.cpu().numpy() == 0x0F).all()
    geo_engine.ipv4_tcp_batch(d, 2, offsets=_t(off))
    want, _ = pack_contiguous([bytes(w) for w in good], 3)
    assert (d.cpu().numpy() == want).all()  # bytes outside the fields untouched too


def test_ipv4_header_cases(engine, orc):
    cases = wires("ipv4_cases.json")
    buf, off = _pack_wires([c["bytes"] for c in cases], 1)
    ip, tcp, st = engine.ipv4_tcp_batch(_t(buf), 1, offsets=_t(off))
    ip, st = _u16(ip), st.cpu().numpy()
    for i, c in enumerate(cases):
        assert bool(st[i] & 1) == c["parse_ok"], c["tag"]
        if "computed" in c:
            assert ip[i] == c["computed"], c["tag"]
    # and the full outputs equal the oracle in every mode
    for mode in (0, 1, 2):
        d = _t(buf)
        g = engine.ipv4_tcp_batch(d, mode, offsets=_t(off))
        hb = buf.copy()
        w = orc.ipv4_tcp_batch(hb, len(cases), mode, offsets=off)
        assert (_u16(g[0]) == w[0]).all() and (_u16(g[1]) == w[1]).all()
        assert (g[2].cpu().numpy() == w[2]).all()
        assert (d.cpu().numpy() == hb).all()


def test_router_fixture(engine):
    cases = wires("router_cases.json")
    buf, off = _pack_wires([c["wire"] for c in cases], 2)
    d = _t(buf)
    st = engine.router_ttl_batch(d, offsets=_t(off)).cpu().numpy()
    assert st.tolist() == [int(c["forwarded"]) for c in cases]
    want, _ = _pack_wires([c["out"] for c in cases], 2)
    assert (d.cpu().numpy() == want).all()


# -------------------------------------------------- workload generators ---
def test_workload_generators_match_spec(engine, orc):
    import torch

    for pos0, nb in [(0, 4096), (3, 1001), (8, 17), (12345, 70000)]:
        t = torch.empty(nb, dtype=torch.uint8, device="cuda:0")
        engine.fill_bytes(t, 0x10710004, pos0)
        assert (t.cpu().numpy() == orc.fill_bytes(0x10710004, pos0, nb)).all()
    init = engine.pseudo_inits(1000, 0x10710000, seg_len=1500, index0=77)
    assert (_u32(init) == orc.pseudo_inits(0x10710000, 1000, length=1500, index0=77)).all()
    d = torch.zeros(50 * 1500, dtype=torch.uint8, device="cuda:0")
    engine.ipv4_tcp_headers(d, 50, 1500, 1500, 0x10710002)
    h = np.zeros(50 * 1500, dtype=np.uint8)
    for i in range(50):
        orc.ipv4_tcp_headers(0x10710002, i, 1500, h[i * 1500:])
    assert (d.cpu().numpy() == h).all()


# --------------------------------- BASELINE configs at FULL size vs reference
def _gen_bytes(engine, nbytes, seed):
    import torch

    t = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    return engine.fill_bytes(t, seed)


@pytest.mark.parametrize("k", ["0", "3", "5"])
def test_config_fixed_stride_full_size(engine, k):
    import torch

    g = golden("configs.json")[k]
    n, stride, seed = g["n"], g["stride"], g["seed"]
    data = _gen_bytes(engine, n * stride, seed)
    init = engine.pseudo_inits(n, seed, seg_len=g["seg_len"])
    out = _u16(engine.checksum_batch(data, n=n, stride=stride, seg_len=g["seg_len"], init=init))
    del data
    torch.cuda.empty_cache()
    assert out[:64].tolist() == g["out_head"]
    assert _sha(out) == g["out_sha256"]


def test_config4_mixed_full_size(engine):
    import torch

    from tcpip_network_protocol_stack_amd.engine import mixed_offsets

    g = golden("configs.json")["4"]
    n, seed = g["n"], g["seed"]
    off = mixed_offsets(n, seed)
    assert int(off[-1]) == 10292782014
    data = _gen_bytes(engine, int(off[-1]), seed)
    doff = _t(off.view(np.int64))
    init = engine.pseudo_inits(n, seed, offsets=doff)
    out = _u16(engine.checksum_batch(data, offsets=doff, init=init))
    del data
    torch.cuda.empty_cache()
    assert out[:64].tolist() == g["out_head"]
    assert _sha(out) == g["out_sha256"]


def test_config2_ipv4_full_size(engine):
    g = golden("configs.json")["2"]
    n, L, seed = g["n"], g["stride"], g["seed"]
    d = _gen_bytes(engine, n * L, seed)
    engine.ipv4_tcp_headers(d, n, L, L, seed)
    ip, tcp, st = engine.ipv4_tcp_batch(d, 0, n=n, stride=L, dgram_len=L)
    assert _sha(_u16(ip)) == g["ipck_sha256"] and _sha(_u16(tcp)) == g["tcpck_sha256"]
    info = engine.dispatch_info()  # fixed-length MTU datagrams: 7 loads per lane (ipv4_fixed_geometry)
    assert (info["kernel"], info["lps"], info["unroll"]) == ("ipv4", 16, 7), info
    engine.ipv4_tcp_batch(d, 2, n=n, stride=L, dgram_len=L)
    assert _sha(d.cpu().numpy()) == g["patched_sha256"]
    _, _, st = engine.ipv4_tcp_batch(d, 1, n=n, stride=L, dgram_len=L)
    assert (st.cpu().numpy() == 0x0F).all()


def test_config7_router_full_size(engine):
    """Router step over config 2's datagrams with ttl = i % 4 (half dropped at
    ttl 0 / 1) vs the reference's parse + Router step (configs.json "7")."""
    import torch

    g = golden("configs.json")["7"]
    n, L, seed = g["n"], g["stride"], g["seed"]
    d = _gen_bytes(engine, n * L, seed)
    engine.ipv4_tcp_headers(d, n, L, L, seed)
    d.view(n, L)[:, 8] = (torch.arange(n, device=d.device) % 4).to(torch.uint8)
    engine.ipv4_tcp_batch(d, 2, n=n, stride=L, dgram_len=L)  # both checksums for the new ttl
    st = engine.router_ttl_batch(d, n=n, stride=L, dgram_len=L).cpu().numpy()
    assert int(st.sum()) == g["forwarded"] and _sha(st) == g["fwd_sha256"]
    assert _sha(d.cpu().numpy()) == g["out_sha256"]


def test_corruption_detection_full_size(engine, orc):
    # inject one random bit flip per datagram of config 2; every flip outside
    # the IPv4 reserved flag bit (which the reference does not represent,
    # ipv4_header.cpp:78) must be rejected, exactly as the oracle says
    import torch

    g = golden("configs.json")["2"]
    n, L, seed = g["n"], g["stride"], g["seed"]
    d = _gen_bytes(engine, n * L, seed)
    engine.ipv4_tcp_headers(d, n, L, L, seed)
    engine.ipv4_tcp_batch(d, 2, n=n, stride=L, dgram_len=L)
    rng = np.random.default_rng(7)
    bit = rng.integers(0, L * 8, n)
    pos = torch.from_numpy(np.arange(n) * L + bit // 8).to("cuda:0")
    mask = torch.from_numpy((1 << (bit % 8)).astype(np.uint8)).to("cuda:0")
    d[pos] = d[pos] ^ mask
    _, _, st = engine.ipv4_tcp_batch(d, 1, n=n, stride=L, dgram_len=L)
    st = st.cpu().numpy()
    reserved = bit == 6 * 8 + 7
    assert (st[~reserved] != 0x0F).all()
    assert (st[reserved] == 0x0F).all()
    host = d.cpu().numpy()
    sample = rng.choice(n, 512, replace=False)
    for i in sample:
        _, _, s, _ = orc.ipv4_tcp(host[i * L:(i + 1) * L].tobytes(), 1)
        assert s == st[i]


# ------------------------------------------------ host-memory variants ---
def test_host_path_checksum(engine, orc):
    rng = np.random.default_rng(5)
    n, L = 200_000, 1500  # > one 32 MiB staging slot: every slot of the pipeline, several times
    buf = rng.integers(0, 256, n * L, dtype=np.uint8)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    got = engine.checksum_batch_host(buf, n, stride=L, seg_len=L, init=init)
    assert (got == orc.checksum_batch(buf, n, stride=L, seg_len=L, init=init, threads=8)).all()
    lens = rng.integers(0, 9000, 20_000)
    segs = [rng.integers(0, 256, int(x), dtype=np.uint8).tobytes() for x in lens]
    b2, off = pack_contiguous(segs, 1)
    got = engine.checksum_batch_host(b2, len(segs), offsets=off)
    assert (got == orc.checksum_batch(b2, len(segs), offsets=off)).all()


@pytest.mark.parametrize("pinned", [False, True])
def test_host_path_segments_longer_than_a_slot(engine, orc, pinned):
    """InternetChecksum::add takes any length (util/tools/checksum.h:20-28):
    segments longer than the 32 MiB staging slot go through the slots as
    pieces (raw sums with the piece's parity, summed mod 2^32, then value()).
    A 100 MiB segment between short ones (odd start, odd length), the
    reference's uint32 wrap case (131 076 x 0xFF -> 0x0001) and a fixed-stride
    batch of 40 MiB segments, all against the oracle."""
    import torch

    rng = np.random.default_rng(77)
    big = rng.integers(0, 256, (100 << 20) + 3, dtype=np.uint8).tobytes()
    segs = [b"\x01\x02\x03", big, b"", rng.integers(0, 256, 1501, dtype=np.uint8).tobytes(), b"\xff" * 131076,
            rng.integers(0, 256, (33 << 20) + 1, dtype=np.uint8).tobytes(), b"\x7f"]
    buf, off = pack_contiguous(segs, 1)
    h = torch.empty(buf.size, dtype=torch.uint8, pin_memory=pinned).numpy()
    h[:] = buf
    init = np.array([0, 0x5FFFA, 7, 0xFFFFFFFF, 0, 0x10000, 1], dtype=np.uint32)
    got = engine.checksum_batch_host(h, len(segs), offsets=off, init=init)
    want = orc.checksum_batch(buf, len(segs), offsets=off, init=init)
    assert (got == want).all(), (got, want)
    assert got[4] == orc.checksum_batch(np.frombuffer(b"\xff" * 131076, np.uint8), 1, offsets=[0, 131076])[0]
    wrap = [c for c in golden("checksum_kat.json")["cases"] if c["tag"] == "fill" and c["len"] == 131076
            and c["fill"] == 0xFF]
    if wrap:
        assert got[4] == wrap[0]["value"] == 0x0001
    n, L = 3, 40 << 20
    data = rng.integers(0, 256, n * L + 5, dtype=np.uint8)
    got = engine.checksum_batch_host(data, n, stride=L + 1, seg_len=L - 1)
    assert (got == orc.checksum_batch(data, n, stride=L + 1, seg_len=L - 1)).all()


def test_host_path_ipv4_datagram_longer_than_a_slot_is_an_error(engine):
    from tcpip_network_protocol_stack_amd._lib import IcsumError

    big = np.zeros((33 << 20), dtype=np.uint8)
    with pytest.raises(IcsumError):
        engine.ipv4_tcp_batch_host(big, 1, 1, offsets=np.array([0, big.size], dtype=np.uint64))


def test_host_path_ipv4_patch(engine, orc):
    cases = wires("tcp_wrap.json", {"wrap"})
    good = [bytes.fromhex(c["wire"]) for c in cases]
    junk = [w[:10] + b"\0\0" + w[12:36] + b"\0\0" + w[38:] for w in good]
    buf, off = pack_contiguous(junk, 0)
    ip, tcp, st = engine.ipv4_tcp_batch_host(buf, len(junk), 2, offsets=off)
    want, _ = pack_contiguous(good, 0)
    assert (buf == want).all() and (st == 0x0F).all()


def _random_datagrams(rng, n):
    """Raw datagrams with every header shape the fused kernel must handle:
    hlen 0-15 (options, and < 5), lengths 0-1600 incl. < 20 and < 40 bytes,
    ver != 4, random flags (reserved bit), proto, TCP data offsets, and a
    third of them carrying valid checksums (patched by the oracle)."""
    from oracle import oracle as orc

    segs = []
    for i in range(n):
        L = int(rng.choice([0, 1, 19, 20, 21, 39, 40, 41, 57, 60, 61]) if i % 5 == 0 else rng.integers(20, 1600))
        b = bytearray(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        if L >= 20:
            hlen = int(rng.choice([5, 5, 5, 6, 8, 15, 4, 0]))
            ver = 4 if rng.random() < 0.9 else int(rng.integers(0, 16))
            b[0] = (ver << 4) | hlen
            b[2:4] = int(rng.integers(0, 65536) if rng.random() < 0.2 else L).to_bytes(2, "big")
            b[9] = 6 if rng.random() < 0.9 else int(rng.integers(0, 256))
            t = 4 * max(hlen, 5)
            if t + 12 < L:
                b[t + 12] = (int(rng.integers(0, 16)) if rng.random() < 0.2 else 5) << 4
            if i % 3 == 0:
                _, _, _, b = orc.ipv4_tcp(bytes(b), 2)  # valid checksums
                b = bytearray(b)
        segs.append(bytes(b))
    return segs


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("lead", [0, 3])
def test_host_path_ipv4_random_all_modes(engine, orc, pinned, lead):
    """ics_ipv4_tcp_batch_host on every header shape, from pageable and from
    page-locked memory: PATCH from host memory writes the two fields on the
    host from a device COMPUTE pass; bytes, checksums and statuses must equal
    the oracle's (and the device-memory path's) in every mode."""
    import torch

    rng = np.random.default_rng(131 + lead)
    segs = _random_datagrams(rng, 1500)
    buf, off = pack_contiguous(segs, lead)
    for mode in (0, 1, 2):
        h = torch.empty(buf.size, dtype=torch.uint8, pin_memory=pinned).numpy()
        h[:] = buf
        ip, tcp, st = engine.ipv4_tcp_batch_host(h, len(segs), mode, offsets=off)
        hb = buf.copy()
        w = orc.ipv4_tcp_batch(hb, len(segs), mode, offsets=off)
        assert (ip == w[0]).all(), mode
        assert (tcp == w[1]).all(), mode
        assert (st == w[2]).all(), mode
        assert (h == hb).all(), mode


@pytest.mark.parametrize("pinned", [False, True])
def test_host_path_ipv4_patch_fixed_stride(engine, orc, pinned):
    """Fixed-stride PATCH from host memory over more datagrams than one
    staging slot holds (several chunks in flight)."""
    import torch

    n, L = 40_000, 1500
    data = orc.fill_bytes(0x10710002, 0, n * L)
    h = torch.empty(n * L, dtype=torch.uint8, pin_memory=pinned).numpy()
    h[:] = data
    for i in range(0, n, 7):  # some headers with options, some with short hlen
        h[i * L] = 0x40 | (5 + (i % 3) * 2 if i % 2 else i % 5)
    hb = h.copy()
    ip, tcp, st = engine.ipv4_tcp_batch_host(h, n, 2, stride=L, dgram_len=L)
    w = orc.ipv4_tcp_batch(hb, n, 2, stride=L, dgram_len=L)
    assert (ip == w[0]).all() and (tcp == w[1]).all() and (st == w[2]).all()
    assert (h == hb).all()


@pytest.mark.parametrize("mix", ["acks", "mtu", "bimodal", "ackheavy", "ackjumbo", "long"])
def test_ipv4_offsets_plan_cache(engine, orc, mix):
    """Raw-datagram offsets batches of >= 16 Ki datagrams take their geometry
    from the plan cached for the offsets buffer (4-lane groups for ACK
    batches, 8-lane groups for ACK-heavy MTU mixes, 16 x 4 otherwise; the plan
    kernels run behind the first and every 64th call): 20 calls in COMPUTE and
    VERIFY, the same buffer rewritten with another mix, then PATCH; every
    output and the patched bytes equal the oracle's."""
    import torch

    rng = np.random.default_rng(0x1B + len(mix))
    n = 20_000
    offs = []
    for m in (mix, "mtu" if mix != "mtu" else "acks"):
        lens = _mix_lengths(rng, n, m).astype(np.uint64)
        o = np.zeros(n + 1, dtype=np.uint64)
        o[1:] = np.cumsum(lens)
        offs.append(o + 3)  # unaligned starts
    buf = rng.integers(0, 256, int(max(o[-1] for o in offs)) + 16, dtype=np.uint8)  # holds both mixes
    for o in offs:  # IPv4/TCP headers that parse: ver 4, hlen 5, len, proto 6, TCP data offset 5
        s, ln = o[:-1].astype(np.int64), np.diff(o)
        buf[s], buf[s + 2], buf[s + 3] = 0x45, (ln >> 8).astype(np.uint8), (ln & 255).astype(np.uint8)
        buf[s + 6], buf[s + 8], buf[s + 9], buf[s + 32] = 0x40, 64, 6, 0x50
    dbuf = _t(buf)
    doff = _t(offs[0])
    for k, off in enumerate(offs):
        if k:
            torch.cuda.synchronize()
            doff.copy_(_t(off))
        for mode in (0, 1):
            want = orc.ipv4_tcp_batch(buf.copy(), n, mode, offsets=off)
            for call in range(20):
                ip, tcp, st = engine.ipv4_tcp_batch(dbuf, mode, offsets=doff)
                assert (_u16(ip) == want[0]).all(), (mix, k, mode, call)
                assert (_u16(tcp) == want[1]).all(), (mix, k, mode, call)
                assert (st.cpu().numpy() == want[2]).all(), (mix, k, mode, call)
    hb = buf.copy()
    orc.ipv4_tcp_batch(hb, n, 2, offsets=offs[1])
    engine.ipv4_tcp_batch(dbuf, 2, offsets=doff)
    assert (dbuf.cpu().numpy() == hb).all(), mix


@pytest.mark.parametrize("lead", [0, 1, 2, 3])
def test_ipv4_tcp_random_all_modes(geo_engine, orc, lead):
    rng = np.random.default_rng(97 + lead)
    segs = _random_datagrams(rng, 1500)
    buf, off = pack_contiguous(segs, lead)
    for mode in (0, 1, 2):
        d = _t(buf)
        ip, tcp, st = geo_engine.ipv4_tcp_batch(d, mode, offsets=_t(off))
        hb = buf.copy()
        w = orc.ipv4_tcp_batch(hb, len(segs), mode, offsets=off)
        assert (_u16(ip) == w[0]).all(), mode
        assert (_u16(tcp) == w[1]).all(), mode
        assert (st.cpu().numpy() == w[2]).all(), mode
        assert (d.cpu().numpy() == hb).all(), mode


def test_router_random(engine, orc):
    rng = np.random.default_rng(5)
    segs = _random_datagrams(rng, 3000)
    # valid headers with every ttl, so forwarding happens and ttl 0/1 drop
    for i in range(0, len(segs), 2):
        if len(segs[i]) >= 20:
            b = bytearray(segs[i])
            b[0] = 0x45
            b[8] = i % 256
            _, _, _, b = orc.ipv4_tcp(bytes(b), 2)
            segs[i] = b
    buf, off = pack_contiguous(segs, 1)
    d = _t(buf)
    st = engine.router_ttl_batch(d, offsets=_t(off)).cpu().numpy()
    hb = buf.copy()
    want = []
    for i in range(len(segs)):
        s, o = int(off[i]), int(off[i + 1])
        f, out = orc.router_ttl(hb[s:o].tobytes())
        hb[s:o] = np.frombuffer(out, dtype=np.uint8)
        want.append(f)
    assert st.tolist() == want
    assert (d.cpu().numpy() == hb).all()
    assert 0 < sum(want) < len(segs)


@pytest.mark.parametrize("stride", [1500, 1502, 64])
def test_router_fixed_stride(engine, orc, stride):
    """Fixed-stride router batches: stride 1500 / 64 keep every header
    dword-aligned (one 8-byte store rewrites wire bytes 4..11), 1502 mixes
    aligned and 2-byte-offset headers (narrow stores); reserved flag bits set
    on some headers must be dropped, every ttl from 0 to 255 appears."""
    rng = np.random.default_rng(7)
    n = 2048
    buf = rng.integers(0, 256, n * stride, dtype=np.uint8)
    for i in range(n):
        b = bytearray(buf[i * stride:(i + 1) * stride].tobytes())
        b[0] = 0x45
        b[2], b[3] = stride >> 8, stride & 0xFF
        b[6] = (b[6] | 0x80) if i % 3 == 0 else (b[6] & 0x7F)
        b[8] = i % 256
        if i % 5 != 4:  # every fifth header keeps a wrong checksum (dropped)
            _, _, _, b = orc.ipv4_tcp(bytes(b), 2)
        buf[i * stride:(i + 1) * stride] = np.frombuffer(bytes(b), dtype=np.uint8)
    d = _t(buf)
    st = engine.router_ttl_batch(d, n=n, stride=stride, dgram_len=stride).cpu().numpy()
    hb = buf.copy()
    want = []
    for i in range(n):
        f, out = orc.router_ttl(hb[i * stride:(i + 1) * stride].tobytes())
        hb[i * stride:(i + 1) * stride] = np.frombuffer(out, dtype=np.uint8)
        want.append(f)
    assert st.tolist() == want
    assert (d.cpu().numpy() == hb).all()
    assert 0 < sum(want) < n


@pytest.mark.parametrize("run", [0, 1, 3, 10])
def test_xcd_block_order_is_a_permutation(run, orc):
    """block_order (k_checksum / k_ipv4_tcp) only permutes blocks: every run
    length (2^run blocks; 0 = hardware order), on grids that are not a multiple of the 8-block window, gives the
    oracle's result for every segment (a dropped or doubled block would leave
    outputs unwritten / wrong).  The order is process-wide, so the default is
    restored afterwards."""
    import torch

    gen = _engine_with({"xcd_remap": run})
    eng = next(gen)
    try:
        rng = np.random.default_rng(run + 7)
        for n, L in ((16 * 8 * 3 + 5, 1500), (16 * 8 * 1024 + 16 * 3 + 1, 576), (4 * 8 * 7 + 3, 9000)):
            data = rng.integers(0, 256, n * L, dtype=np.uint8)
            init = rng.integers(0, 1 << 20, n, dtype=np.uint32)
            got = _u16(eng.checksum_batch(_t(data), n=n, stride=L, seg_len=L, init=_t(init)))
            want = orc.checksum_batch(data, n, stride=L, seg_len=L, init=init)
            assert (got == want).all(), (run, n, L, np.flatnonzero(got != want)[:8])
        # the fused datagram kernel uses the same order
        n, L = 16 * 8 * 3 + 9, 1500
        dg = torch.empty(n * L, dtype=torch.uint8, device="cuda:0")
        eng.fill_bytes(dg, 0x10710002)
        eng.ipv4_tcp_headers(dg, n, L, L, 0x10710002)
        ip, tcp, st = eng.ipv4_tcp_batch(dg, 0, n=n, stride=L, dgram_len=L)
        host = dg.cpu().numpy().copy()
        want_ip, want_tcp, want_st = orc.ipv4_tcp_batch(host, n, 0, stride=L, dgram_len=L)
        assert (_u16(ip) == want_ip).all() and (_u16(tcp) == want_tcp).all()
        assert (st.cpu().numpy() == want_st).all()
    finally:
        torch.cuda.synchronize()
        eng.close()
        next(_engine_with({"xcd_remap": 10})).close()  # restore the default order


@pytest.mark.parametrize("segs", [1, 2, 4, 8])
def test_dense_fixed_stride_kernel(segs, orc):
    """k_checksum_dense (stride == seg_len in {32, 64, 128}, aligned, no
    parity array) at every SEGS: u16 values and raw u32 sums, with and without
    inits, on batch sizes that leave partial waves and blocks; unsupported
    (seg_len, segs) pairs fall back to the general kernels and must agree too."""
    gen = _engine_with({"dense_segs": segs})
    eng = next(gen)
    try:
        rng = np.random.default_rng(100 + segs)
        for L in (32, 64, 128):
            for n in (1, 15, 16 * segs + 3, 4096 * 3 + 7):
                data = rng.integers(0, 256, n * L, dtype=np.uint8)
                init = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
                d = _t(data)
                for ini in (None, init):
                    got = _u16(eng.checksum_batch(d, n=n, stride=L, seg_len=L, init=None if ini is None else _t(ini)))
                    want = orc.checksum_batch(data, n, stride=L, seg_len=L, init=ini)
                    assert (got == want).all(), (segs, L, n, ini is None)
                got = _u32(eng.sum_batch(d, n=n, stride=L, seg_len=L, init=_t(init)))
                assert (got == orc.sum_batch(data, n, stride=L, seg_len=L, init=init)).all(), (segs, L, n)
        # an all-0xFF batch: sums near the fold boundary, value() of 0xFFFF inits
        n, L = 5000, 64
        data = np.full(n * L, 0xFF, dtype=np.uint8)
        init = np.full(n, 0xFFFF, dtype=np.uint32)
        got = _u16(eng.checksum_batch(_t(data), n=n, stride=L, seg_len=L, init=_t(init)))
        assert (got == orc.checksum_batch(data, n, stride=L, seg_len=L, init=init)).all()
    finally:
        import torch

        torch.cuda.synchronize()
        eng.close()


def test_force_hook_rejects_unknown_keys():
    """ICSUM_FORCE (the test hook) fails ics_create on a key it does not know
    or a value out of range, so a mistyped hook cannot silently test the
    default path instead."""
    from tcpip_network_protocol_stack_amd._lib import IcsumError

    for bad in ("lps=16,bogus=1", "twoclass=12", "wrap_passes=3", "bin_plan", "lps=x"):
        with pytest.raises(IcsumError, match="ICSUM_FORCE"):
            next(_engine_with_raw(bad))
    eng = next(_engine_with({"lps": 16, "unroll": 8, "mode": 3}))
    eng.close()


def _engine_with_raw(spec):
    import os

    from tcpip_network_protocol_stack_amd.engine import Engine

    os.environ["ICSUM_FORCE"] = spec
    try:
        yield Engine(0)
    finally:
        os.environ.pop("ICSUM_FORCE", None)
