"""GPU: batches of more than 2^32 SEGMENTS — the segment-count analogue of
test_gpu_offsets_4g.py's byte offsets.  The API takes a 64-bit count; the
kernels cap their grids at 2^22 blocks and grid-stride over the rest, so a
segment or group index built in 32 bits anywhere would wrap past 2^32 and
silently recompute (or skip) segments.  The plan cache and the binning passes
take at most 2^32 - 1 segments by design (a larger batch runs one launch at
the unknown-mix geometry); this module pins that path too.

* 2^32 + 2^20 + 3 one-byte segments at stride 1 (4 GiB of bytes, 8 GiB of u16
  outputs): the plain checksum through the automatic choice (one lane per
  segment) and forced 16- / 64-lane line grids and the small-segment body,
  and the unfolded sums; every output checked on the device (a single byte
  is a high byte: value = ~(b << 8)).
* 2^32 + 1001 packed offsets (34 GiB), all segments empty except eight —
  placed at 0, 1, 2^31 - 1, 2^31, 2^32 - 1, 2^32, 2^32 + 1 and the last —
  holding real datagrams: the plain checksum (automatic, forced one lane,
  forced 16-lane, the tile launch), IPv4/TCP VERIFY (automatic, one lane,
  the tile launch) and the router.
  Every empty segment must give the oracle's value for an empty segment, the
  eight the oracle's values for their bytes.

Outputs start as sentinel patterns.  Bar: bit-exact."""
import numpy as np
import pytest

from conftest import engine_with, force_id

pytestmark = pytest.mark.gpu

N1 = (1 << 32) + (1 << 20) + 3
N2 = (1 << 32) + 1001
PICK = (0, 1, (1 << 31) - 1, 1 << 31, (1 << 32) - 1, 1 << 32, (1 << 32) + 1, N2 - 1)
SEED = 0x4D1B0C00
CHUNK = 1 << 28


def _torch():
    import torch

    return torch


@pytest.fixture(scope="module")
def ones(engine):
    """N1 + 16 seeded random bytes: N1 one-byte segments at stride 1."""
    torch = _torch()
    t = torch.empty(N1 + 16, dtype=torch.uint8, device="cuda:0")
    engine.fill_bytes(t, SEED)
    torch.cuda.synchronize()
    yield t
    del t
    torch.cuda.empty_cache()


FIXED_FORCE = [None, {"lps": 16, "unroll": 8, "mode": 3}, {"lps": 64, "unroll": 8, "mode": 3},
               {"lps": 4, "unroll": 2, "mode": 2, "segs": 2}]


@pytest.fixture(scope="module", params=FIXED_FORCE, ids=lambda f: force_id(f or {}))
def feng(request):
    for eng in engine_with(request.param):
        eng.forced = request.param
        yield eng


def _check_one_byte(data, out, raw):
    """out[i] == ~(b_i << 8) (folded u16) or b_i << 8 (raw u32), all N1 of them."""
    torch = _torch()
    for a in range(0, N1, CHUNK):
        b = min(N1, a + CHUNK)
        x = data[a:b].to(torch.int32) << 8
        if raw:
            assert torch.equal(out[a:b], x), a
        else:
            assert torch.equal(out[a:b].to(torch.int32) & 0xFFFF, 0xFFFF - x), a


def test_fixed_stride_one_byte_segments_past_2p32(feng, ones):
    torch = _torch()
    out = feng.checksum_batch(ones, n=N1, stride=1, seg_len=1)
    torch.cuda.synchronize()
    assert out.numel() == N1
    _check_one_byte(ones, out, raw=False)
    if feng.forced:
        info = feng.dispatch_info()
        assert (info["lps"], info["unroll"]) == (feng.forced["lps"], feng.forced["unroll"]), info
    del out
    torch.cuda.empty_cache()


def test_fixed_stride_sums_past_2p32(engine, ones):
    torch = _torch()
    out = engine.sum_batch(ones, n=N1, stride=1, seg_len=1)
    torch.cuda.synchronize()
    _check_one_byte(ones, out, raw=True)
    del out
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def sparse(engine):
    """(bytes, offsets, datagrams): N2 segments, empty except at PICK."""
    from test_gpu_parity import _random_datagrams

    torch = _torch()
    rng = np.random.default_rng(0x4D1B)
    segs = [s for s in _random_datagrams(rng, 64) if len(s) >= 20][:len(PICK)]
    assert len(segs) == len(PICK)
    off = torch.zeros(N2 + 1, dtype=torch.int64, device="cuda:0")
    for j, s in zip(PICK, segs):
        off[j + 1:] += len(s)
    buf = np.frombuffer(b"".join(segs) + b"\0" * 64, dtype=np.uint8).copy()
    data = torch.from_numpy(buf).cuda()
    torch.cuda.synchronize()
    assert int(off[-1]) == sum(len(s) for s in segs)
    yield data, off, segs
    del off, data
    torch.cuda.empty_cache()


def _only_picks_differ(t, empty_value):
    """Every element equals empty_value except possibly those at PICK; returns t[PICK] on the host."""
    torch = _torch()
    picks = torch.tensor(PICK, dtype=torch.int64, device=t.device)
    got = t[picks].cpu().numpy()
    for a in range(0, t.numel(), CHUNK):
        b = min(t.numel(), a + CHUNK)
        bad = t[a:b] != empty_value
        inside = [p - a for p in PICK if a <= p < b]
        if inside:
            bad[torch.tensor(inside, dtype=torch.int64, device=t.device)] = False
        assert not bool(bad.any()), f"an empty segment in [{a}, {b}) differs"
    return got


OFF_FORCE = [None, {"lps": 1, "unroll": 4, "mode": 4}, {"lps": 16, "unroll": 8, "mode": 3}, {"tile": 1}]


@pytest.fixture(scope="module", params=OFF_FORCE, ids=lambda f: force_id(f or {}))
def oeng(request):
    yield from engine_with(request.param)


def test_offsets_mostly_empty_past_2p32(oeng, orc, sparse):
    torch = _torch()
    data, off, segs = sparse
    out = oeng.checksum_batch(data, offsets=off)
    torch.cuda.synchronize()
    assert out.numel() == N2
    empty = int(orc.checksum_batch(np.zeros(1, np.uint8), 1, stride=0, seg_len=0)[0])
    got = _only_picks_differ(out, np.int16(np.uint16(empty)).item())
    want = [int(orc.checksum_batch(np.frombuffer(s, np.uint8), 1, stride=len(s), seg_len=len(s))[0]) for s in segs]
    assert [int(v) for v in got.view(np.uint16)] == want
    del out
    torch.cuda.empty_cache()


IPV4_FORCE = [None, {"lps": 1, "unroll": 4, "mode": 4}, {"tile": 1}]


@pytest.fixture(scope="module", params=IPV4_FORCE, ids=lambda f: force_id(f or {}))
def veng(request):
    yield from engine_with(request.param)


def test_ipv4_verify_mostly_empty_past_2p32(veng, orc, sparse):
    torch = _torch()
    data, off, segs = sparse
    ip = torch.empty(N2, dtype=torch.int16, device="cuda:0")
    tcp = torch.empty(N2, dtype=torch.int16, device="cuda:0")
    st = torch.empty(N2, dtype=torch.uint8, device="cuda:0")
    for t, v in ((ip, 0x5A5A), (tcp, 0x5A5A), (st, 0x5A)):
        t.fill_(np.int16(np.uint16(v)).item() if t.dtype == torch.int16 else v)
    veng.ipv4_tcp_batch(data, 1, n=N2, offsets=off, ip_ck=ip, tcp_ck=tcp, status=st)
    torch.cuda.synchronize()
    eip, etcp, est, _ = orc.ipv4_tcp(b"", 1)
    gip = _only_picks_differ(ip, np.int16(np.uint16(eip)).item()).view(np.uint16)
    gtcp = _only_picks_differ(tcp, np.int16(np.uint16(etcp)).item()).view(np.uint16)
    gst = _only_picks_differ(st, est)
    for k, s in enumerate(segs):
        wip, wtcp, wst, _ = orc.ipv4_tcp(s, 1)
        assert (int(gip[k]), int(gtcp[k]), int(gst[k])) == (wip, wtcp, wst), (k, PICK[k])
    del ip, tcp, st
    torch.cuda.empty_cache()


def test_router_mostly_empty_past_2p32(engine, orc, sparse):
    torch = _torch()
    data, off, segs = sparse
    work = data.clone()
    st = torch.full((N2,), 0x5A, dtype=torch.uint8, device="cuda:0")
    engine.router_ttl_batch(work, n=N2, offsets=off, status=st)
    torch.cuda.synchronize()
    est, _ = orc.router_ttl(b"")
    gst = _only_picks_differ(st, est)
    got = work.cpu().numpy()
    pos = 0
    for k, s in enumerate(segs):
        wst, wbytes = orc.router_ttl(s)
        assert int(gst[k]) == wst, (k, PICK[k])
        assert got[pos:pos + len(s)].tobytes() == wbytes, (k, PICK[k])
        pos += len(s)
    del work, st
    torch.cuda.empty_cache()
