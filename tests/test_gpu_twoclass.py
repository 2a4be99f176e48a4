"""GPU parity of the two-class launches of packed offsets batches
(k_checksum_twoclass and k_ipv4_twoclass: short segments one per lane, long
ones 16 lanes each from a per-wave LDS list), forced on every offsets batch
with the `twoclass` test hook at both wave loads AUTO uses (16 and 32
segments per wave), against the golden KATs and the oracle.  AUTO reaches
them through a cached plan of a short-heavy mix; the last test checks that
path.  Bar: bit-exact."""
import numpy as np
import pytest

from helpers import kat_cases, pack_contiguous
from conftest import engine_with, force_id
from test_gpu_parity import _t, _u16, _u32

pytestmark = pytest.mark.gpu

TWO_FORCE = [{"twoclass": 8}, {"twoclass": 16}, {"twoclass": 32}]


@pytest.fixture(scope="module", params=TWO_FORCE, ids=force_id)
def two_csum(request):
    yield from engine_with(request.param)


def _sentinel(n, dtype):
    """Output buffer pre-filled with a pattern: an output the kernels never
    write shows up (a fresh allocation may hold an earlier call's results)."""
    import torch

    return torch.full((n,), 0x5A5A if dtype == torch.int16 else 0x5A5A5A5A, dtype=dtype, device="cuda:0")


def _check(eng, orc, buf, off, rng, tag=""):
    import torch

    n = off.size - 1
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    out = eng.checksum_batch(_t(buf), offsets=_t(off), init=_t(init), out=_sentinel(n, torch.int16))
    assert (_u16(out) == orc.checksum_batch(buf, n, offsets=off, init=init)).all(), tag
    out0 = eng.checksum_batch(_t(buf), offsets=_t(off), out=_sentinel(n, torch.int16))  # init NULL = 0
    assert (_u16(out0) == orc.checksum_batch(buf, n, offsets=off)).all(), tag
    odd = rng.integers(0, 2, n).astype(np.uint8)
    sums = eng.sum_batch(_t(buf), offsets=_t(off), init=_t(init), odd=_t(odd), out=_sentinel(n, torch.int32))
    assert (_u32(sums) == orc.sum_batch(buf, n, offsets=off, init=init, odd=odd)).all(), tag


def test_twoclass_kats(two_csum):
    # every KAT (lengths 0-257, inits, whole segments, the 131076-byte 0xFF
    # wrap) at four alignments of the first byte
    cases = kat_cases({"rfc1071", "len", "init", "whole", "fill"})
    segs = [b"".join(p) for _, p, _, _ in cases]
    init = np.array([c[0] for c in cases], dtype=np.uint32)
    for lead in (0, 1, 6, 15):
        buf, off = pack_contiguous(segs, lead)
        out = two_csum.checksum_batch(_t(buf), offsets=_t(off), init=_t(init),
                                         out=_sentinel(len(cases), __import__("torch").int16))
        assert _u16(out).tolist() == [c[2] for c in cases], f"lead={lead}"


def test_twoclass_split_pieces_chain(two_csum):
    # add(vector<string>) with parity carried across pieces (checksum.h:44-59)
    cases = kat_cases({"split"})
    maxp = max(len(p) for _, p, _, _ in cases)
    sums = np.array([c[0] for c in cases], dtype=np.uint32)
    odd = np.zeros(len(cases), dtype=np.uint8)
    for k in range(maxp):
        segs = [p[k] if k < len(p) else b"" for _, p, _, _ in cases]
        buf, off = pack_contiguous(segs, 1)
        sums = _u32(two_csum.sum_batch(_t(buf), offsets=_t(off), init=_t(sums), odd=_t(odd))).copy()
        odd ^= np.array([len(x) & 1 for x in segs], dtype=np.uint8)
    assert _u16(two_csum.fold_batch(_t(sums))).tolist() == [c[2] for c in cases]


def test_twoclass_mixed(two_csum, orc):
    # lengths over every bin, zero-length segments, a few long ones
    rng = np.random.default_rng(0xF1A7)
    n = 6000
    edges = [0, 1, 15, 16, 17, 143, 144, 145, 1919, 1920, 4096, 8191, 8192, 8193]
    lens = rng.choice([40, 64, 100, 576, 1500, 3000, 9000, 40000], n) + rng.integers(-7, 8, n)
    lens[: len(edges)] = edges
    lens[len(edges)::101] = 0
    segs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
    for lead in (0, 5, 15):
        buf, off = pack_contiguous(segs, lead)
        _check(two_csum, orc, buf, off, rng, f"lead={lead}")


def test_twoclass_tiny_segments(two_csum, orc):
    # 0-20 byte segments: several cuts inside one 16-byte chunk, more than 64
    # cuts per tile (the cut loop's further rounds)
    rng = np.random.default_rng(0x7111)
    n = 40_000
    lens = rng.integers(0, 21, n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    off += 3
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    _check(two_csum, orc, buf, off, rng)


def test_twoclass_long_segments(two_csum, orc):
    # segments far longer than a share (3 MiB, 1 MiB + 1) between short ones:
    # their pieces come from many waves
    rng = np.random.default_rng(0x10E6)
    lens = rng.integers(0, 3000, 400)
    lens[50] = 3 << 20
    lens[51] = (1 << 20) + 1
    lens[399] = 700_001
    off = np.zeros(lens.size + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    off += 9
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    _check(two_csum, orc, buf, off, rng)


@pytest.mark.parametrize("lens", [[0] * 100, [0], [1], [15], [16], [17], [100_000], [0, 0, 5, 0, 0],
                                  [8192] * 3, [8191, 1, 8192, 0]])
def test_twoclass_edge_batches(two_csum, orc, lens):
    # all-empty batches (every output = the folded init), single segments,
    # segments that end exactly on tile boundaries
    rng = np.random.default_rng(len(lens) * 7 + sum(lens))
    for lead in (0, 11):
        off = np.zeros(len(lens) + 1, dtype=np.uint64)
        off[1:] = np.cumsum(lens)
        off += lead
        buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
        _check(two_csum, orc, buf, off, rng, f"lead={lead}")


def test_twoclass_bimodal_large(two_csum, orc):
    # ACK-sized + MSS-sized segments interleaved (a TCP receive mix)
    rng = np.random.default_rng(0xACC)
    n = 150_000
    lens = np.where(rng.random(n) < 0.5, 40, 1460) + rng.integers(0, 4, n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    off += 1
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    out = two_csum.checksum_batch(_t(buf), offsets=_t(off), out=_sentinel(n, __import__("torch").int16))
    assert (_u16(out) == orc.checksum_batch(buf, n, offsets=off)).all()


def test_twoclass_config4_full_size(two_csum):
    # BASELINE config 4 at full size (10.3 GB: positions past 2^31 and 2^32)
    # against the reference's digest, into a sentinel-filled output
    import hashlib

    import torch

    from conftest import golden
    from tcpip_network_protocol_stack_amd.engine import mixed_offsets

    g = golden("configs.json")["4"]
    n, seed = g["n"], g["seed"]
    off = mixed_offsets(n, seed)
    data = two_csum.fill_bytes(torch.empty(int(off[-1]), dtype=torch.uint8, device="cuda:0"), seed)
    doff = _t(off.view(np.int64))
    init = two_csum.pseudo_inits(n, seed, offsets=doff)
    out = _u16(two_csum.checksum_batch(data, offsets=doff, init=init, out=_sentinel(n, torch.int16)))
    del data
    torch.cuda.empty_cache()
    assert out[:64].tolist() == g["out_head"]
    assert hashlib.sha256(out.tobytes()).hexdigest() == g["out_sha256"]


@pytest.fixture(scope="module", params=[{"twoclass": 32}, {"twoclass": 16}, {"twoclass": 8}], ids=force_id)
def two_engine(request):
    yield from engine_with(request.param)


@pytest.mark.parametrize("mix", ["bimodal", "ackheavy", "tricky"])
def test_ipv4_twoclass_vs_oracle(two_engine, orc, mix):
    """Raw IPv4/TCP datagram batches through the two-class fused launch
    (k_ipv4_twoclass: the block's <= 64-byte datagrams one per lane on one
    wave, the rest 16 lanes each claimed by every wave; forced with the
    twoclass hook): COMPUTE,
    VERIFY and PATCH against the oracle, patched bytes included.  "tricky"
    adds short (< 20 B), 64/65-byte edge, option-carrying and corrupted
    datagrams."""
    rng = np.random.default_rng(0x1F0 + len(mix))
    n = 20_000
    ack = lambda p: np.where(rng.random(n) < p, 40, 1460) + rng.integers(0, 4, n)  # noqa: E731
    lens = {"bimodal": lambda: ack(0.5), "ackheavy": lambda: ack(0.75),
            "tricky": lambda: rng.choice([0, 7, 19, 20, 36, 37, 38, 39, 40, 41, 42, 63, 64, 65, 100, 1460, 1500],
                                         n)}[mix]()
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    off += 3
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    s, ln = off[:-1].astype(np.int64), np.diff(off).astype(np.int64)
    ok = ln >= (36 if mix == "tricky" else 40)  # 36..39: TCP parts of 16..19 bytes (the checksum field cut)
    s, ln = s[ok], ln[ok]
    buf[s], buf[s + 2], buf[s + 3] = 0x45, (ln >> 8).astype(np.uint8), (ln & 255).astype(np.uint8)
    buf[s + 6], buf[s + 8], buf[s + 9] = 0x40, 64, 6
    buf[s[ln > 32] + 32] = 0x50
    if mix == "tricky":
        buf[s[::7]] = 0x46  # options (hlen 6)
        buf[s[::11] + 25] ^= 0x10  # corrupted TCP bytes
    for mode in (0, 1, 2):
        hb = buf.copy()
        want = orc.ipv4_tcp_batch(hb, n, mode, offsets=off)
        d = _t(buf)
        ip, tcp, st = two_engine.ipv4_tcp_batch(d, mode, offsets=_t(off))
        assert (_u16(ip) == want[0]).all(), (mix, mode)
        assert (_u16(tcp) == want[1]).all(), (mix, mode)
        assert (st.cpu().numpy() == want[2]).all(), (mix, mode)
        assert (d.cpu().numpy() == hb).all(), (mix, mode)  # PATCH wrote what the oracle wrote


def test_auto_reaches_twoclass_from_cached_plan(engine, orc):
    """The default dispatch: a short-heavy receive mix (3/4 ACKs among MTU
    segments) plans on its first call and runs the two-class launches from
    the cached plan on the next ones — checksum and fused VERIFY — with the
    oracle's results every time."""
    rng = np.random.default_rng(0x2C1A)
    n = 70_000
    lens = np.where(rng.random(n) < 0.75, 40, 1460) + rng.integers(0, 4, n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    s, ln = off[:-1].astype(np.int64), lens.astype(np.int64)
    buf[s], buf[s + 2], buf[s + 3] = 0x45, (ln >> 8).astype(np.uint8), (ln & 255).astype(np.uint8)
    buf[s + 9], buf[s + 32] = 6, 0x50
    d, do = _t(buf), _t(off)
    want = orc.checksum_batch(buf, n, offsets=off)
    want_v = orc.ipv4_tcp_batch(buf.copy(), n, 1, offsets=off)
    kinds = []
    for call in range(3):
        assert (_u16(engine.checksum_batch(d, offsets=do)) == want).all(), call
        __import__("torch").cuda.synchronize()
        kinds.append(engine.dispatch_info()["kernel"])
        ip, tcp, st = engine.ipv4_tcp_batch(d, 1, offsets=do)
        assert (_u16(ip) == want_v[0]).all() and (_u16(tcp) == want_v[1]).all(), call
        assert (st.cpu().numpy() == want_v[2]).all(), call
        info = engine.dispatch_info()
        kinds.append(info["kernel"])
        if call:  # 3/4 short datagrams: the wide block lists, 32 per wave (kIpv4TwoClassWide16)
            assert info["unroll"] == 32, info
    assert kinds[2:] == ["twoclass", "ipv4_twoclass"] * 2, kinds
