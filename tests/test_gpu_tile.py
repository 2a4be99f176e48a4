"""GPU parity of the tile launch of offsets batches (k_span: one wave per 63
consecutive segments, the span's bytes streamed whole in 4 KiB windows, each
segment's sums = F(hi) - F(lo) of the running prefix), forced on every
offsets batch with the `tile` test hook — short last spans, one-segment
batches, spans of empty segments, offsets past 2^31 and 2^32 (config 4 at
full size) and the grid-stride form that more spans than one grid holds take
(reached with a capped grid, the span_blocks hook): checksum (u16,
raw u32 sums with carried parity), the fused IPv4/TCP kernel in all three
modes (PATCH's in-place stores racing a neighbouring span's boundary chunk:
every F of a span comes from one copy of each window, so those bytes cancel),
the in-place wrap and the headers-apart wrap, against the golden KATs, the
reference's own wrap output (tests/golden/tcp_wrap.json) and the oracle.
Bar: bit-exact."""
import numpy as np
import pytest

from conftest import engine_with, force_id
from helpers import kat_cases, pack_contiguous, wires
from test_gpu_parity import _t, _u16, _u32
from test_gpu_twoclass import _check, _sentinel

pytestmark = pytest.mark.gpu

# the tile launch (k_span) on every offsets batch: 63 segments per wave (or
# the plan's span size), one, and an odd size that leaves short last spans;
# then the grid-stride instantiation (k_span<..., STRIDE=true>, which a batch
# of more spans than 2^24 blocks hold takes) with the grid capped to a few
# blocks by the span_blocks hook, so each wave runs many spans in turn and
# reuses its LDS windows and register sets across them
TILE_FORCE = [{"tile": 1}, {"tile": 1, "span_segs": 1}, {"tile": 1, "span_segs": 7},
              {"tile": 1, "span_segs": 1, "span_blocks": 3}, {"tile": 1, "span_segs": 7, "span_blocks": 5}]


@pytest.fixture(scope="module", params=TILE_FORCE, ids=force_id)
def tile_eng(request):
    yield from engine_with(request.param)


def _assert_tile(eng):
    """the tile launch (k_span) ran, at the forced span size if any"""
    info = eng.dispatch_info()
    assert info["kernel"] == "tile", info
    S = getattr(eng, "forced", {}).get("span_segs", 0)
    assert info["lps"] == S if S else 1 <= info["lps"] <= 63, info


def test_tile_kats(tile_eng):
    # every KAT (lengths 0-257, inits, whole segments, the 131076-byte 0xFF
    # wrap: nine windows) at four alignments of the first byte
    import torch

    cases = kat_cases({"rfc1071", "len", "init", "whole", "fill"})
    segs = [b"".join(p) for _, p, _, _ in cases]
    init = np.array([c[0] for c in cases], dtype=np.uint32)
    for lead in (0, 1, 6, 15):
        buf, off = pack_contiguous(segs, lead)
        out = tile_eng.checksum_batch(_t(buf), offsets=_t(off), init=_t(init), out=_sentinel(len(cases), torch.int16))
        _assert_tile(tile_eng)
        assert _u16(out).tolist() == [c[2] for c in cases], f"lead={lead}"


def test_tile_split_pieces_chain(tile_eng):
    # add(vector<string>) with parity carried across pieces (checksum.h:44-59)
    cases = kat_cases({"split"})
    maxp = max(len(p) for _, p, _, _ in cases)
    sums = np.array([c[0] for c in cases], dtype=np.uint32)
    odd = np.zeros(len(cases), dtype=np.uint8)
    for k in range(maxp):
        segs = [p[k] if k < len(p) else b"" for _, p, _, _ in cases]
        buf, off = pack_contiguous(segs, 1)
        sums = _u32(tile_eng.sum_batch(_t(buf), offsets=_t(off), init=_t(sums), odd=_t(odd))).copy()
        odd ^= np.array([len(x) & 1 for x in segs], dtype=np.uint8)
    assert _u16(tile_eng.fold_batch(_t(sums))).tolist() == [c[2] for c in cases]


def test_tile_mixed(tile_eng, orc):
    # lengths around every window / chunk edge, zero-length segments, long ones
    rng = np.random.default_rng(0x711E)
    n = 6000
    edges = [0, 1, 15, 16, 17, 143, 144, 145, 1919, 1920, 16383, 16384, 16385, 40000]
    lens = rng.choice([40, 64, 100, 576, 1500, 3000, 9000, 40000], n) + rng.integers(-7, 8, n)
    lens[: len(edges)] = edges
    lens[len(edges)::101] = 0
    segs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
    for lead in (0, 5, 15):
        buf, off = pack_contiguous(segs, lead)
        _check(tile_eng, orc, buf, off, rng, f"lead={lead}")
        _assert_tile(tile_eng)


def test_tile_tiny_segments(tile_eng, orc):
    # 0-20 byte segments: several segment starts inside one 16-byte chunk
    rng = np.random.default_rng(0x7112)
    n = 40_000
    lens = rng.integers(0, 21, n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    off += 3
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    _check(tile_eng, orc, buf, off, rng)


def test_tile_long_segments(tile_eng, orc):
    # segments of many windows (3 MiB = 192 windows, 1 MiB + 1) between short ones
    rng = np.random.default_rng(0x10E7)
    lens = rng.integers(0, 3000, 400)
    lens[50] = 3 << 20
    lens[51] = (1 << 20) + 1
    lens[399] = 700_001
    off = np.zeros(lens.size + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    off += 9
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    _check(tile_eng, orc, buf, off, rng)


@pytest.mark.parametrize("lens", [[0] * 100, [0], [1], [15], [16], [17], [100_000], [0, 0, 5, 0, 0],
                                  [16384] * 3, [16383, 1, 16384, 0], [32768, 0, 0]])
def test_tile_edge_batches(tile_eng, orc, lens):
    # all-empty batches, single segments, segments ending exactly on window edges
    rng = np.random.default_rng(len(lens) * 13 + sum(lens))
    for lead in (0, 11, 16):
        off = np.zeros(len(lens) + 1, dtype=np.uint64)
        off[1:] = np.cumsum(lens)
        off += lead
        buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
        _check(tile_eng, orc, buf, off, rng, f"lead={lead}")


def _dgram_batch(rng, n, mix):
    ack = lambda p: np.where(rng.random(n) < p, 40, 1460) + rng.integers(0, 4, n)  # noqa: E731
    lens = {"bimodal": lambda: ack(0.5), "ackheavy": lambda: ack(0.75),
            "tricky": lambda: rng.choice([0, 7, 19, 20, 21, 39, 40, 41, 57, 63, 64, 65, 100, 1460, 1500], n)}[mix]()
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    off += 3
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    s, ln = off[:-1].astype(np.int64), np.diff(off).astype(np.int64)
    ok = ln >= 40
    s, ln = s[ok], ln[ok]
    buf[s], buf[s + 2], buf[s + 3] = 0x45, (ln >> 8).astype(np.uint8), (ln & 255).astype(np.uint8)
    buf[s + 6], buf[s + 8], buf[s + 9], buf[s + 32] = 0x40, 64, 6, 0x50
    if mix == "tricky":
        buf[s[::7]] = 0x46  # options (hlen 6)
        buf[s[::13]] = 0x4F  # hlen 15: the TCP part starts past most short datagrams' ends
        buf[s[::11] + 25] ^= 0x10  # corrupted TCP bytes
    return buf, off


@pytest.mark.parametrize("mix", ["bimodal", "ackheavy", "tricky"])
def test_tile_ipv4_vs_oracle(tile_eng, orc, mix):
    """COMPUTE, VERIFY and PATCH of raw IPv4/TCP datagram batches through the
    tile launch, patched bytes included; "tricky" has datagrams under 20 and
    40 bytes, options, header lengths past the datagram's end and corrupted
    bytes, and with 1- or 7-datagram tiles their boundary chunks hold the
    neighbours' checksum fields that PATCH rewrites."""
    rng = np.random.default_rng(0x7F0 + len(mix))
    n = 20_000
    buf, off = _dgram_batch(rng, n, mix)
    for mode in (0, 1, 2):
        hb = buf.copy()
        want = orc.ipv4_tcp_batch(hb, n, mode, offsets=off)
        d = _t(buf)
        ip, tcp, st = tile_eng.ipv4_tcp_batch(d, mode, offsets=_t(off))
        _assert_tile(tile_eng)
        assert (_u16(ip) == want[0]).all(), (mix, mode)
        assert (_u16(tcp) == want[1]).all(), (mix, mode)
        assert (st.cpu().numpy() == want[2]).all(), (mix, mode)
        assert (d.cpu().numpy() == hb).all(), (mix, mode)  # PATCH wrote what the oracle wrote


def _msgs_from_cases(cases):
    from test_gpu_wrap import _msgs_from_cases as f

    return f(cases)


@pytest.mark.parametrize("lead", [0, 1, 2, 3])
def test_tile_wrap_reproduces_reference_wire_bytes(tile_eng, lead):
    import torch

    cases = wires("tcp_wrap.json", {"wrap"})
    segs = [b"\xee" * 40 + bytes.fromhex(c["wire"][80:80 + 2 * c["payload_len"]]) for c in cases]
    buf, off = pack_contiguous(segs, lead)
    d = torch.from_numpy(buf).cuda()
    dm = torch.from_numpy(_msgs_from_cases(cases).view(np.uint8).copy()).cuda()
    ip = torch.empty(len(cases), dtype=torch.int16, device="cuda")
    tcp = torch.empty(len(cases), dtype=torch.int16, device="cuda")
    tile_eng.tcp_wrap_batch(d, dm, n=len(cases), offsets=_t(off), ip_ck=ip, tcp_ck=tcp)
    _assert_tile(tile_eng)
    got = d.cpu().numpy()
    for i, c in enumerate(cases):
        assert got[off[i]:off[i + 1]].tobytes().hex() == c["wire"], i
    assert [int(x) for x in _u16(ip)] == [c["ip_cksum"] for c in cases]
    assert (got[:lead] == 0xA5).all()  # nothing before the first datagram touched


def test_tile_wrap_random_vs_oracle(tile_eng, orc):
    import torch

    from test_gpu_wrap import _oracle_wire, _random_batch

    rng = np.random.default_rng(2025)
    segs, m = _random_batch(rng, 12000)
    segs.append(b"\0" * 40 + rng.integers(0, 256, 70000, dtype=np.uint8).tobytes())  # len field wraps mod 2^16
    m = np.concatenate([m, m[:1]])
    segs += [b"\x5a" * 39, b"", b"\x5b" * 17]  # shorter than 40: untouched
    m = np.concatenate([m, m[:3]])
    want = _oracle_wire(orc, segs[:-3], m[:-3]) + segs[-3:]
    buf, off = pack_contiguous(segs, 1)
    d = torch.from_numpy(buf).cuda()
    ip = torch.empty(len(segs), dtype=torch.int16, device="cuda")
    tile_eng.tcp_wrap_batch(d, torch.from_numpy(m.view(np.uint8).copy()).cuda(), n=len(segs), offsets=_t(off),
                            ip_ck=ip)
    got = d.cpu().numpy()
    for i, w in enumerate(want):
        assert got[off[i]:off[i + 1]].tobytes() == w, i
    assert (_u16(ip)[-3:] == 0).all()


def test_tile_config4_full_size():
    """BASELINE config 4 at full size (10.3 GB: offsets past 2^31 and 2^32)
    through the tile launch, against the reference's digest."""
    import hashlib

    import torch

    from conftest import golden
    from tcpip_network_protocol_stack_amd.engine import mixed_offsets

    for eng in engine_with({"tile": 1}):
        g = golden("configs.json")["4"]
        n, seed = g["n"], g["seed"]
        off = mixed_offsets(n, seed)
        data = eng.fill_bytes(torch.empty(int(off[-1]), dtype=torch.uint8, device="cuda:0"), seed)
        doff = _t(off.view(np.int64))
        init = eng.pseudo_inits(n, seed, offsets=doff)
        out = _u16(eng.checksum_batch(data, offsets=doff, init=init, out=_sentinel(n, torch.int16)))
        _assert_tile(eng)
        del data
        torch.cuda.empty_cache()
        assert out[:64].tolist() == g["out_head"]
        assert hashlib.sha256(out.tobytes()).hexdigest() == g["out_sha256"]


@pytest.fixture(scope="module", params=TILE_FORCE, ids=force_id)
def tile_apart(request):
    yield from engine_with(request.param)


@pytest.mark.parametrize("lead", [0, 3])
def test_tile_wrap_headers_apart(tile_apart, orc, lead):
    """ics_tcp_wrap_headers as one tile launch (payload sums, the 40-byte
    headers stored to their array as each tile's contiguous block): the
    reference's wire bytes for every golden wrap case, and random payloads
    (0..1460 bytes) against the oracle."""
    import torch

    from test_gpu_wrap import _oracle_wire, _random_batch

    cases = wires("tcp_wrap.json", {"wrap"})
    pays = [bytes.fromhex(c["wire"][80:80 + 2 * c["payload_len"]]) for c in cases]
    buf, off = pack_contiguous(pays, lead)
    hd = torch.empty(len(cases) * 40, dtype=torch.uint8, device="cuda")
    dm = torch.from_numpy(_msgs_from_cases(cases).view(np.uint8).copy()).cuda()
    tile_apart.tcp_wrap_headers(_t(buf), dm, hd, n=len(cases), offsets=_t(off))
    _assert_tile(tile_apart)
    h = hd.cpu().numpy()
    for i, c in enumerate(cases):
        assert h[40 * i:40 * i + 40].tobytes().hex() == c["wire"][:80], i
    rng = np.random.default_rng(77 + lead)
    segs, m = _random_batch(rng, 5000)
    want = _oracle_wire(orc, segs, m)
    buf, off = pack_contiguous([s[40:] for s in segs], lead)
    hd = torch.empty(len(segs) * 40, dtype=torch.uint8, device="cuda")
    tile_apart.tcp_wrap_headers(_t(buf), torch.from_numpy(m.view(np.uint8).copy()).cuda(), hd, n=len(segs),
                                offsets=_t(off))
    h = hd.cpu().numpy()
    for i, w in enumerate(want):
        assert h[40 * i:40 * i + 40].tobytes() == w[:40], i


def test_auto_reaches_tile_from_cached_plan(engine, orc):
    """The default dispatch: an offsets batch of variable-length datagrams
    (40..1040 bytes: 0..1000-byte payloads, the transmit side's mix) above
    the tile threshold plans on its first call and runs the tile launch from
    the cached plan on the next ones — checksum, VERIFY and the headers-apart
    wrap — with the oracle's results every time; an MTU-only batch keeps the
    per-segment launches."""
    import torch

    from tcpip_network_protocol_stack_amd.engine import TCP_MSG_DTYPE

    rng = np.random.default_rng(0x7A0)
    n = 140_000
    lens = 40 + rng.integers(0, 1001, n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    s = off[:-1].astype(np.int64)
    buf[s], buf[s + 2], buf[s + 3] = 0x45, (lens >> 8).astype(np.uint8), (lens & 255).astype(np.uint8)
    buf[s + 6], buf[s + 8], buf[s + 9], buf[s + 32] = 0x40, 64, 6, 0x50
    orc.ipv4_tcp_batch(buf, n, 2, offsets=off)  # valid checksums
    d, do = _t(buf), _t(off)
    want = orc.checksum_batch(buf, n, offsets=off)
    want_v = orc.ipv4_tcp_batch(buf.copy(), n, 1, offsets=off)
    kinds = []
    for call in range(3):
        assert (_u16(engine.checksum_batch(d, offsets=do)) == want).all(), call
        kinds.append(engine.dispatch_info()["kernel"])
        ip, tcp, st = engine.ipv4_tcp_batch(d, 1, offsets=do)
        assert (_u16(ip) == want_v[0]).all() and (_u16(tcp) == want_v[1]).all(), call
        assert (st.cpu().numpy() == want_v[2]).all(), call
        kinds.append(engine.dispatch_info()["kernel"])
    assert kinds[2:] == ["tile", "tile"] * 2, kinds
    # headers apart: payloads of the same lengths minus 40
    m = np.zeros(n, dtype=TCP_MSG_DTYPE)
    for f, hi in (("src", 2**32), ("dst", 2**32), ("seqno", 2**32), ("ackno", 2**32), ("src_port", 2**16),
                  ("dst_port", 2**16), ("window", 2**16)):
        m[f] = rng.integers(0, hi, n, dtype=np.uint64)
    m["flags"], m["ttl"] = 0x10, 128
    pay = [buf[int(off[i]) + 40:int(off[i + 1])].tobytes() for i in range(n)]
    pb, poff = pack_contiguous(pay, 0)
    dm = torch.from_numpy(m.view(np.uint8).copy()).cuda()
    got = []
    for call in range(3):
        hd = torch.empty(n * 40, dtype=torch.uint8, device="cuda")
        engine.tcp_wrap_headers(_t(pb), dm, hd, n=n, offsets=_t(poff))
        got.append((engine.dispatch_info()["kernel"], hd.cpu().numpy()))
    assert got[2][0] == "tile" and got[0][0] != "tile", [g[0] for g in got]
    assert (got[0][1] == got[1][1]).all() and (got[1][1] == got[2][1]).all()  # every path: the same headers
    # ... and those are the reference's: a sample against the oracle's wrap
    from test_gpu_wrap import _oracle_wire

    idx = rng.choice(n, 300, replace=False)
    want_w = _oracle_wire(orc, [b"\0" * 40 + pay[i] for i in idx], m[idx])
    for k, i in enumerate(idx):
        assert got[2][1][40 * i:40 * i + 40].tobytes() == want_w[k][:40], i
    # MTU-sized datagrams: the per-segment launch stays
    lm = np.full(n, 1500)
    offm = np.zeros(n + 1, dtype=np.uint64)
    offm[1:] = np.cumsum(lm)
    bm = rng.integers(0, 256, int(offm[-1]) + 16, dtype=np.uint8)
    for call in range(3):
        engine.checksum_batch(_t(bm), offsets=_t(offm))
    assert engine.dispatch_info()["kernel"] != "tile"
