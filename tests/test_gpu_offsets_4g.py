"""GPU: every kernel family on batches whose byte offsets cross 2^31 and 2^32.

One device buffer of 4 GiB + 80 MiB.  Fixed-stride batches start at its first
byte and run to its end, so segment starts i * stride pass both boundaries
(strides chosen so one segment straddles each boundary and, for 64 and 1024,
one starts exactly on it); packed-offsets batches are placed so that a segment
straddles a boundary or starts exactly on it, with short and long segments on
both sides.  Every family is run through the C-ABI — the plain checksum and
the unfolded sums under the tiny, small, dense, two-class and line-grid
kernels and under every binned plan; the fused IPv4/TCP kernel in COMPUTE,
VERIFY and PATCH (one lane, 4/8/16/64-lane groups, the two-class launch, the
plan-cache path); the device wrap in place and with the headers apart, one
and two passes; the tile launch (k_span) for the checksum, the fused kernel
and both wraps; the router step — into sentinel-filled outputs, and compared
with the oracle (oracle/icsum_oracle.c) on the bytes around each boundary and
at both ends of the batch.  The bug class this pins: a 64-bit offset or start
built from a 32-bit value somewhere (round 2: a sign-extended readlane in the
since-removed flat dispatch).  Bar: bit-exact."""
import numpy as np
import pytest

from conftest import engine_with, force_id
from helpers import oracle_wrap_wire

pytestmark = pytest.mark.gpu

B31, B32 = 1 << 31, 1 << 32
BIG = B32 + (80 << 20)
SEED = 0x4D1B0000
BOUNDS = (B31, B32)


def _torch():
    import torch

    return torch


def _dev(a):
    """numpy -> device tensor (unsigned words as same-width signed views)."""
    torch = _torch()
    a = np.ascontiguousarray(a)
    sig = {np.dtype(np.uint16): np.int16, np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64}
    if a.dtype in sig:
        a = a.view(sig[a.dtype])
    return torch.from_numpy(a.copy()).cuda()


def _u(t, dt):
    return t.cpu().numpy().view(dt)


def _sentinel(n, dtype):
    torch = _torch()
    v = {torch.int16: 0x5A5A, torch.int32: 0x5A5A5A5A, torch.uint8: 0x5A}[dtype]
    return torch.full((n,), v, dtype=dtype, device="cuda:0")


@pytest.fixture(scope="module")
def big(engine):
    """The 4 GiB + 80 MiB buffer of seeded random bytes (read-only for the
    checksum tests; the tests that write make their own copy)."""
    torch = _torch()
    t = torch.empty(BIG, dtype=torch.uint8, device="cuda:0")
    engine.fill_bytes(t, SEED)
    torch.cuda.synchronize()
    yield t
    del t
    torch.cuda.empty_cache()


def _fresh(engine, seed=SEED):
    torch = _torch()
    t = torch.empty(BIG, dtype=torch.uint8, device="cuda:0")
    engine.fill_bytes(t, seed)
    return t


def _host(t, a, b):
    return t[a:b].cpu().numpy()


# ---------------------------------------------------------- batch shapes ----
def _fixed_windows(n, stride):
    """index ranges [i0, i1) of the segments around each boundary, plus both ends"""
    out = [(0, min(n, 48)), (max(0, n - 48), n)]
    for b in BOUNDS:
        c = b // stride
        out.append((max(0, c - 300), min(n, c + 300)))
    return out


MIX_LENS = {
    "mix": [0, 1, 15, 16, 17, 40, 63, 64, 65, 100, 576, 1460, 1500, 2999, 9001],
    "ack": [0, 1, 20, 39, 40, 41, 44, 52, 56, 60],
}


def _offsets_at(rng, bnd, how, lens_pool, n=20_000):
    """Packed offsets of n segments placed so that segment n//2 straddles the
    boundary `bnd` (how="straddle": it starts 5 bytes below it) or starts
    exactly on it (how="on")."""
    lens = rng.choice(lens_pool, n).astype(np.uint64)
    lens[n // 2] = max(int(lens[n // 2]), 1500 if max(lens_pool) > 100 else 40)
    rel = np.zeros(n + 1, dtype=np.uint64)
    rel[1:] = np.cumsum(lens)
    start = bnd - int(rel[n // 2]) - (5 if how == "straddle" else 0)
    return rel + np.uint64(start)


def _window(t, off):
    """host copy of the batch's bytes and its offsets relative to that copy"""
    a = int(off[0])
    return _host(t, a, int(off[-1]) + 16), off - np.uint64(a)


# ---------------------------------------------- a1-a4: plain checksums ------
FIXED = [(1500, 1500), (1024, 1000), (9000, 9000), (40, 40), (64, 64), (72, 64), (130, 128)]


@pytest.mark.parametrize("stride,L", FIXED, ids=[f"{s}x{l}" for s, l in FIXED])
def test_fixed_stride_checksum_across_2g_4g(engine, orc, big, stride, L):
    """Default dispatch of fixed-stride batches spanning the whole buffer:
    (16,8) line grid, 1000/1024 (segments starting on the boundaries), the
    64-lane grid, the one-lane tiny kernel (40 B), the dense kernel (64 B
    aligned) and the small-segment kernel (64 B in 72 B strides), plus raw
    sums with parity carried in."""
    torch = _torch()
    n = (BIG - L) // stride + 1
    assert (n - 1) * stride + L > B32
    init = engine.pseudo_inits(n, SEED, seg_len=L)
    out = engine.checksum_batch(big, n=n, stride=stride, seg_len=L, init=init, out=_sentinel(n, torch.int16))
    odd = torch.randint(0, 2, (n,), dtype=torch.uint8, device="cuda:0")
    sums = engine.sum_batch(big, n=n, stride=stride, seg_len=L, init=init, odd=odd, out=_sentinel(n, torch.int32))
    torch.cuda.synchronize()
    for i0, i1 in _fixed_windows(n, stride):
        data = _host(big, i0 * stride, (i1 - 1) * stride + L)
        ini = _u(init[i0:i1], np.uint32)
        want = orc.checksum_batch(data, i1 - i0, stride=stride, seg_len=L, init=ini)
        assert (_u(out[i0:i1], np.uint16) == want).all(), (stride, L, i0)
        want_s = orc.sum_batch(data, i1 - i0, stride=stride, seg_len=L, init=ini, odd=_u(odd[i0:i1], np.uint8))
        assert (_u(sums[i0:i1], np.uint32) == want_s).all(), (stride, L, i0)


OFF_FORCE = [None,
             {"bin": 1, "bin_plan": 0}, {"bin": 1, "bin_plan": 1}, {"bin": 1, "bin_plan": 2},
             {"bin": 1, "bin_plan": 3}, {"bin": 1, "bin_plan": 0, "last_bin_lps": 32},
             {"lps": 1, "unroll": 4, "mode": 4},
             {"lps": 4, "unroll": 1, "mode": 2, "segs": 2}, {"lps": 4, "unroll": 2, "mode": 2, "segs": 2},
             {"lps": 8, "unroll": 2, "mode": 2, "segs": 2},
             {"lps": 16, "unroll": 8, "mode": 3}, {"lps": 64, "unroll": 8, "mode": 3},
             {"twoclass": 8}, {"twoclass": 16}, {"twoclass": 32},
             {"tile": 1}]


@pytest.fixture(scope="module", params=OFF_FORCE, ids=lambda f: force_id(f or {}))
def feng(request):
    yield from engine_with(request.param)


@pytest.mark.parametrize("mix", ["mix", "ack"])
def test_offsets_checksum_across_2g_4g(feng, orc, big, mix):
    """Packed-offsets batches straddling / starting on 2^31 and 2^32 under
    every forced kernel and binned plan (and the default dispatch, called
    three times: miss, then the cached plan)."""
    torch = _torch()
    rng = np.random.default_rng(0xC4 + len(mix))
    for bnd in BOUNDS:
        for how in ("straddle", "on"):
            off = _offsets_at(rng, bnd, how, MIX_LENS[mix])
            n = off.size - 1
            data, rel = _window(big, off)
            init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
            odd = rng.integers(0, 2, n).astype(np.uint8)
            want = orc.checksum_batch(data, n, offsets=rel, init=init)
            want_s = orc.sum_batch(data, n, offsets=rel, init=init, odd=odd)
            doff, dinit, dodd = _dev(off), _dev(init), _dev(odd)
            for call in range(3):
                out = feng.checksum_batch(big, offsets=doff, init=dinit, out=_sentinel(n, torch.int16))
                assert (_u(out, np.uint16) == want).all(), (bnd, how, call, np.flatnonzero(_u(out, np.uint16) != want)[:5])
                s = feng.sum_batch(big, offsets=doff, init=dinit, odd=dodd, out=_sentinel(n, torch.int32))
                assert (_u(s, np.uint32) == want_s).all(), (bnd, how, call)
                torch.cuda.synchronize()


# ------------------------------------------- fused IPv4 + TCP, router -------
def _datagram_window(rng, pool, n=20_000, ttl_mix=False):
    """raw IPv4/TCP datagrams of lengths from `pool` back to back (host):
    version/hlen, total length, DF, ttl, proto, data offset written over
    random bytes (checksum fields random)"""
    lens = rng.choice(pool, n).astype(np.int64)
    lens[n // 2] = max(lens[n // 2], 1500 if max(pool) > 100 else 40)
    rel = np.zeros(n + 1, dtype=np.uint64)
    rel[1:] = np.cumsum(lens)
    buf = rng.integers(0, 256, int(rel[-1]) + 16, dtype=np.uint8)
    s = rel[:-1].astype(np.int64)
    ok = lens >= 40
    s, ln = s[ok], lens[ok]
    buf[s], buf[s + 2], buf[s + 3] = 0x45, (ln >> 8).astype(np.uint8), (ln & 255).astype(np.uint8)
    buf[s + 6], buf[s + 8], buf[s + 9], buf[s + 32] = 0x40, 64, 6, 0x50
    if ttl_mix:
        buf[s + 8] = (np.arange(s.size) % 4).astype(np.uint8)
    buf[s[::13]] = 0x46  # a few option-carrying headers (hlen 6)
    return buf, rel, n


def _place(t, buf, rel, bnd, how):
    """copy a host batch into device buffer t so that datagram n//2 straddles
    `bnd` (or starts on it); returns the absolute offsets"""
    n = rel.size - 1
    start = bnd - int(rel[n // 2]) - (5 if how == "straddle" else 0)
    t[start:start + buf.size].copy_(_torch().from_numpy(buf))
    return rel + np.uint64(start)


IPV4_FORCE = [None, {"twoclass": 32}, {"lps": 1, "unroll": 4, "mode": 4}, {"lps": 4, "unroll": 1, "mode": 2},
              {"lps": 8, "unroll": 2, "mode": 2}, {"lps": 8, "unroll": 8, "mode": 3},
              {"lps": 16, "unroll": 7, "mode": 3}, {"lps": 16, "unroll": 8, "mode": 3},
              {"lps": 64, "unroll": 8, "mode": 3}, {"tile": 1}]
IPV4_MIX = {"ack": [40, 41, 42, 43], "bimodal": [40, 41, 1460, 1500],
            "tricky": [0, 7, 19, 20, 39, 40, 41, 63, 64, 65, 100, 1460, 1500, 9000]}


@pytest.fixture(scope="module", params=IPV4_FORCE, ids=lambda f: force_id(f or {}))
def veng(request):
    yield from engine_with(request.param)


@pytest.mark.parametrize("mix", sorted(IPV4_MIX))
def test_offsets_ipv4_across_2g_4g(veng, orc, mix):
    """ics_ipv4_tcp_batch COMPUTE / VERIFY / PATCH over raw datagrams placed
    across each boundary, patched bytes compared too; the default engine is
    called twice per mode (miss, then its cached plan: one lane per
    datagram for ACKs, the two-class launch for the bimodal mix)."""
    torch = _torch()
    rng = np.random.default_rng(0x4C0 + len(mix))
    t = _fresh(veng)
    for bnd in BOUNDS:
        for how in ("straddle", "on"):
            buf, rel, n = _datagram_window(rng, IPV4_MIX[mix])
            off = _place(t, buf, rel, bnd, how)
            doff = _dev(off)
            for mode in (0, 1, 2):
                for call in range(2):
                    hb = _host(t, int(off[0]), int(off[-1]) + 16)
                    want = orc.ipv4_tcp_batch(hb, n, mode, offsets=rel)
                    ip, tcp, st = veng.ipv4_tcp_batch(t, mode, offsets=doff, ip_ck=_sentinel(n, torch.int16),
                                                      tcp_ck=_sentinel(n, torch.int16), status=_sentinel(n, torch.uint8))
                    torch.cuda.synchronize()
                    tag = (mix, bnd, how, mode, call)
                    assert (_u(ip, np.uint16) == want[0]).all(), tag
                    assert (_u(tcp, np.uint16) == want[1]).all(), tag
                    assert (_u(st, np.uint8) == want[2]).all(), tag
                    assert (_host(t, int(off[0]), int(off[-1]) + 16) == hb).all(), tag  # PATCH: the oracle's bytes
    del t
    torch.cuda.empty_cache()


@pytest.mark.parametrize("L", [1500, 40])
def test_fixed_stride_ipv4_and_router_across_2g_4g(engine, orc, L):
    """Fixed-stride datagrams over the whole buffer (1500 B: 16-lane line
    grid; 40 B: one lane per datagram): COMPUTE, PATCH, VERIFY, then the router
    step, each compared with the oracle around both boundaries and at both
    ends."""
    torch = _torch()
    t = _fresh(engine, SEED + L)
    n = BIG // L
    engine.ipv4_tcp_headers(t, n, L, L, SEED)
    wins = _fixed_windows(n, L)
    before = {w: _host(t, w[0] * L, w[1] * L) for w in wins}
    for mode in (0, 2, 1):
        ip, tcp, st = engine.ipv4_tcp_batch(t, mode, n=n, stride=L, dgram_len=L, ip_ck=_sentinel(n, torch.int16),
                                            tcp_ck=_sentinel(n, torch.int16), status=_sentinel(n, torch.uint8))
        torch.cuda.synchronize()
        for (i0, i1) in wins:
            hb = before[(i0, i1)]
            want = orc.ipv4_tcp_batch(hb, i1 - i0, mode, stride=L, dgram_len=L)
            assert (_u(ip[i0:i1], np.uint16) == want[0]).all(), (L, mode, i0)
            assert (_u(tcp[i0:i1], np.uint16) == want[1]).all(), (L, mode, i0)
            assert (_u(st[i0:i1], np.uint8) == want[2]).all(), (L, mode, i0)
            assert (_host(t, i0 * L, i1 * L) == hb).all(), (L, mode, i0)
            if mode == 1:
                assert (want[2] == 0x0F).all()  # every patched datagram verifies
    # router: ttl 64 everywhere, headers now valid
    st = engine.router_ttl_batch(t, n=n, stride=L, dgram_len=L, status=_sentinel(n, torch.uint8))
    torch.cuda.synchronize()
    for (i0, i1) in wins:
        hb = before[(i0, i1)]
        for i in range(i0, i1):
            f, w = orc.router_ttl(hb[(i - i0) * L:(i - i0 + 1) * L].tobytes())
            assert int(st[i]) == f, (L, i)
            assert _host(t, i * L, (i + 1) * L).tobytes() == w, (L, i)
    del t
    torch.cuda.empty_cache()


def test_offsets_router_across_2g_4g(engine, orc):
    """ics_router_ttl_batch over datagrams with every ttl class placed across
    each boundary (valid checksums first, by the oracle's PATCH)."""
    torch = _torch()
    rng = np.random.default_rng(0x4077)
    t = _fresh(engine)
    for bnd in BOUNDS:
        for how in ("straddle", "on"):
            buf, rel, n = _datagram_window(rng, IPV4_MIX["tricky"], n=4000, ttl_mix=True)
            orc.ipv4_tcp_batch(buf, n, 2, offsets=rel)  # valid header checksums
            off = _place(t, buf, rel, bnd, how)
            st = engine.router_ttl_batch(t, offsets=_dev(off), status=_sentinel(n, torch.uint8)).cpu().numpy()
            got = _host(t, int(off[0]), int(off[-1]) + 16)
            want = []
            for i in range(n):
                a, b = int(rel[i]), int(rel[i + 1])
                f, w = orc.router_ttl(buf[a:b].tobytes())
                buf[a:b] = np.frombuffer(w, dtype=np.uint8)
                want.append(f)
            assert st.tolist() == want, (bnd, how)
            assert (got == buf).all(), (bnd, how)
            assert 0 < sum(want) < n
    del t
    torch.cuda.empty_cache()


# ------------------------------------------------------------ device wrap ---
def _msgs(rng, n):
    from tcpip_network_protocol_stack_amd.engine import TCP_MSG_DTYPE

    m = np.zeros(n, dtype=TCP_MSG_DTYPE)
    for f, hi in (("src", 2**32), ("dst", 2**32), ("seqno", 2**32), ("ackno", 2**32), ("src_port", 2**16),
                  ("dst_port", 2**16), ("window", 2**16), ("id", 2**16)):
        m[f] = rng.integers(0, hi, n, dtype=np.uint64)
    m["flags"] = rng.choice([0x10, 0x12, 0x11, 0x14, 0x02, 0x01, 0x00, 0x17], n)
    m["ttl"] = rng.choice([128, 64, 1, 255], n)
    return m


@pytest.fixture(scope="module", params=[None, {"wrap_passes": 1}, {"wrap_passes": 2}, {"tile": 1}],
                ids=lambda f: force_id(f or {}))
def weng4(request):
    yield from engine_with(request.param)


def test_fixed_stride_wrap_across_2g_4g(weng4, orc):
    """ics_tcp_wrap_batch in place (1040-byte datagrams) and
    ics_tcp_wrap_headers (1000-byte payloads, headers to their own array: two
    passes by default at this size) over the whole buffer; k_tcp_hdr's
    in-place stores rebuild 64-bit starts from two 32-bit shuffles (forced
    two passes)."""
    torch = _torch()
    rng = np.random.default_rng(0x3A9)
    t = _fresh(weng4, SEED + 1)
    for L, apart in ((1040, False), (1000, True)):
        n = BIG // L
        m = _msgs(rng, n)
        dm = torch.from_numpy(m.view(np.uint8).copy()).cuda()
        wins = _fixed_windows(n, L)
        before = {w: _host(t, w[0] * L, w[1] * L) for w in wins}
        ip, tcp = _sentinel(n, torch.int16), _sentinel(n, torch.int16)
        if apart:
            hdrs = torch.full((n * 40,), 0x5A, dtype=torch.uint8, device="cuda:0")
            weng4.tcp_wrap_headers(t, dm, hdrs, n=n, stride=L, payload_len=L, ip_ck=ip, tcp_ck=tcp)
        else:
            weng4.tcp_wrap_batch(t, dm, n=n, stride=L, dgram_len=L, ip_ck=ip, tcp_ck=tcp)
        torch.cuda.synchronize()
        for (i0, i1) in wins:
            hb = before[(i0, i1)]
            ipw, tcpw = _u(ip[i0:i1], np.uint16), _u(tcp[i0:i1], np.uint16)
            for i in range(i0, i1):
                seg = hb[(i - i0) * L:(i - i0 + 1) * L]
                if apart:
                    want = oracle_wrap_wire(orc, seg.tobytes(), m[i])
                    assert _host(hdrs, 40 * i, 40 * i + 40).tobytes() == want[:40], (L, i)
                else:
                    want = oracle_wrap_wire(orc, seg[40:].tobytes(), m[i])
                    assert _host(t, i * L, (i + 1) * L).tobytes() == want, (L, i)
                assert int(ipw[i - i0]) == int.from_bytes(want[10:12], "big"), (L, i)
                assert int(tcpw[i - i0]) == int.from_bytes(want[36:38], "big"), (L, i)
            if apart:
                assert (_host(t, i0 * L, i1 * L) == hb).all()  # payloads untouched
        del dm
    del t
    torch.cuda.empty_cache()


@pytest.mark.parametrize("apart", [False, True])
def test_offsets_wrap_across_2g_4g(weng4, orc, apart):
    """Device wrap of packed-offsets batches placed across each boundary
    (payload lengths 0-1460, ACK-heavy), in place or with the headers apart."""
    torch = _torch()
    rng = np.random.default_rng(0x3AA + apart)
    t = _fresh(weng4, SEED + 2)
    for bnd in BOUNDS:
        for how in ("straddle", "on"):
            n = 6000
            plen = np.where(rng.random(n) < 0.5, 0, rng.integers(0, 1461, n))
            lens = plen + (0 if apart else 40)
            lens[n // 2] = max(lens[n // 2], 1040)
            rel = np.zeros(n + 1, dtype=np.uint64)
            rel[1:] = np.cumsum(lens)
            buf = rng.integers(0, 256, int(rel[-1]) + 16, dtype=np.uint8)
            off = _place(t, buf, rel, bnd, how)
            m = _msgs(rng, n)
            dm = torch.from_numpy(m.view(np.uint8).copy()).cuda()
            if apart:
                hdrs = torch.full((n * 40,), 0x5A, dtype=torch.uint8, device="cuda:0")
                weng4.tcp_wrap_headers(t, dm, hdrs, n=n, offsets=_dev(off))
                hd = hdrs.cpu().numpy()
            else:
                weng4.tcp_wrap_batch(t, dm, n=n, offsets=_dev(off))
            torch.cuda.synchronize()
            got = _host(t, int(off[0]), int(off[-1]) + 16)
            for i in list(range(0, n, 7)) + list(range(n // 2 - 40, n // 2 + 40)) + [n - 1]:
                a, b = int(rel[i]), int(rel[i + 1])
                if apart:
                    want = oracle_wrap_wire(orc, buf[a:b].tobytes(), m[i])
                    assert hd[40 * i:40 * i + 40].tobytes() == want[:40], (bnd, how, i)
                else:
                    want = oracle_wrap_wire(orc, buf[a + 40:b].tobytes(), m[i])
                    assert got[a:b].tobytes() == want, (bnd, how, i)
            if apart:
                assert (got == buf).all()
    del t
    torch.cuda.empty_cache()
