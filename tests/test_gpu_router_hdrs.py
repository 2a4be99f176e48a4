"""GPU: the router step with the forwarded headers apart
(ics_router_ttl_headers, k_router_hdrs).  Router::route decrements the ttl,
recomputes the header checksum and hands send_datagram the datagram, which
serialize() sends as the 20-byte header piece and the payload piece
(/root/reference/src/router/router.cpp:39-66,
util/ipv4_header/ipv4_header.cpp:62-86); here the datagrams are only read and
the forwarded headers go to one array.  Pinned by the reference's own router
cases (tests/golden/router_cases.json), the oracle (random batches, fixed
strides with reserved flag bits and bad checksums, batches across 2^31 and
2^32), and config "7" at full size: the header array spliced back into the
datagrams gives the reference's digest of the in-place router output.
A dropped or unparseable datagram's 20 bytes are zero; the input is never
written.  Bar: bit-exact."""
import hashlib

import numpy as np
import pytest

from conftest import golden
from helpers import pack_contiguous, wires
from test_gpu_parity import _pack_wires, _random_datagrams, _t

pytestmark = pytest.mark.gpu


def _want_hdrs(orc, buf, off):
    """(status, 20 * n header bytes) the reference's router step gives: a
    forwarded datagram's first 20 bytes after the step, zeros otherwise"""
    n = off.size - 1
    st, hd = [], np.zeros(n * 20, dtype=np.uint8)
    for i in range(n):
        a, b = int(off[i]), int(off[i + 1])
        f, out = orc.router_ttl(buf[a:b].tobytes())
        st.append(f)
        if f:
            hd[20 * i:20 * i + 20] = np.frombuffer(out[:20], dtype=np.uint8)
    return st, hd


def _run(engine, d, n, **kw):
    import torch

    hd = torch.full((n * 20,), 0xA5, dtype=torch.uint8, device="cuda:0")  # sentinel: every byte must be written
    st = torch.full((n,), 0x5A, dtype=torch.uint8, device="cuda:0")
    engine.router_ttl_headers(d, n=n, hdrs=hd, status=st, **kw)
    assert engine.dispatch_info()["kernel"] == "router_hdrs"
    return hd.cpu().numpy(), st.cpu().numpy()


def test_router_headers_fixture(engine, orc):
    cases = wires("router_cases.json")
    buf, off = _pack_wires([c["wire"] for c in cases], 2)
    d = _t(buf)
    hd, st = _run(engine, d, len(cases), offsets=_t(off))
    assert st.tolist() == [int(c["forwarded"]) for c in cases]
    for i, c in enumerate(cases):
        want = bytes.fromhex(c["out"])[:20] if c["forwarded"] else bytes(20)
        assert hd[20 * i:20 * i + 20].tobytes() == want, i
    assert (d.cpu().numpy() == buf).all()  # read only


def test_router_headers_random(engine, orc):
    rng = np.random.default_rng(15)
    segs = _random_datagrams(rng, 3000)
    for i in range(0, len(segs), 2):  # valid headers with every ttl: forwarding and ttl 0/1 drops
        if len(segs[i]) >= 20:
            b = bytearray(segs[i])
            b[0] = 0x45 if i % 10 else 0x46  # a few with options (hlen 6: 20 bytes serialized all the same)
            b[6] |= 0x80 if i % 6 == 0 else 0  # reserved flag bit: dropped from the forwarded header
            b[8] = i % 256
            _, _, _, b = orc.ipv4_tcp(bytes(b), 2)
            segs[i] = b
    buf, off = pack_contiguous(segs, 1)
    d = _t(buf)
    hd, st = _run(engine, d, len(segs), offsets=_t(off))
    want_st, want_hd = _want_hdrs(orc, buf, off)
    assert st.tolist() == want_st
    assert (hd == want_hd).all()
    assert (d.cpu().numpy() == buf).all()
    assert 0 < sum(want_st) < len(segs)


@pytest.mark.parametrize("stride", [1500, 1502, 64, 20])
def test_router_headers_fixed_stride(engine, orc, stride):
    rng = np.random.default_rng(stride)
    n = 2051  # not a multiple of a wave's 32 datagrams
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
    hd, st = _run(engine, d, n, stride=stride, dgram_len=stride)
    off = np.arange(n + 1, dtype=np.uint64) * stride
    want_st, want_hd = _want_hdrs(orc, buf, off)
    assert st.tolist() == want_st
    assert (hd == want_hd).all()


def test_router_headers_config7_full_size(engine):
    """Config "7" (config 2's 64 Ki x 1500 B datagrams with ttl = i % 4, half
    dropped): the forwarded headers spliced into the datagrams reproduce the
    reference's digest of the router's output, the status its forwarded set."""
    import torch

    g = golden("configs.json")["7"]
    n, L, seed = g["n"], g["stride"], g["seed"]
    d = engine.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device="cuda:0"), seed)
    engine.ipv4_tcp_headers(d, n, L, L, seed)
    d.view(n, L)[:, 8] = (torch.arange(n, device=d.device) % 4).to(torch.uint8)
    engine.ipv4_tcp_batch(d, 2, n=n, stride=L, dgram_len=L)  # both checksums for the new ttl
    before = hashlib.sha256(d.cpu().numpy().tobytes()).hexdigest()
    hd, st = engine.router_ttl_headers(d, n=n, stride=L, dgram_len=L)
    st = st.cpu().numpy()
    assert int(st.sum()) == g["forwarded"]
    assert hashlib.sha256(st.tobytes()).hexdigest() == g["fwd_sha256"]
    assert hashlib.sha256(d.cpu().numpy().tobytes()).hexdigest() == before  # read only
    fwd = torch.from_numpy(st.astype(bool)).cuda()
    v = d.view(n, L)
    v[fwd, :20] = hd.view(n, 20)[fwd]
    assert hashlib.sha256(d.cpu().numpy().tobytes()).hexdigest() == g["out_sha256"]
    assert (hd.view(n, 20)[~fwd] == 0).all()


def test_router_headers_across_2g_4g(engine, orc):
    """Datagrams with every ttl class placed across 2^31 and 2^32 of a
    4 GiB + 80 MiB buffer (packed offsets)."""
    import torch

    from test_gpu_offsets_4g import BOUNDS, IPV4_MIX, _datagram_window, _dev, _fresh, _place

    rng = np.random.default_rng(0x40A7)
    t = _fresh(engine)
    for bnd in BOUNDS:
        for how in ("straddle", "on"):
            buf, rel, n = _datagram_window(rng, IPV4_MIX["tricky"], n=4000, ttl_mix=True)
            orc.ipv4_tcp_batch(buf, n, 2, offsets=rel)  # valid header checksums
            off = _place(t, buf, rel, bnd, how)
            hd, st = _run(engine, t, n, offsets=_dev(off))
            want_st, want_hd = _want_hdrs(orc, buf, rel)
            assert st.tolist() == want_st, (bnd, how)
            assert (hd == want_hd).all(), (bnd, how)
            assert 0 < sum(want_st) < n
    del t
    torch.cuda.empty_cache()
