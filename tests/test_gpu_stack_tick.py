"""GPU: the shapes one stack tick hands over (VERDICT r3 item 2,
tools/bench_configs.py --only stack) at full size, bit-exact — a receive
batch of 256 Ki raw datagrams, half 40-byte ACKs and half 1500-byte segments
(packed offsets, valid headers with every tenth corrupted), VERIFYed and
COMPUTEd as the TUN loop's unwrap does (tcp_over_ip.cpp:10-36 through
ipv4_header.cpp:9-59 and tcp_segment.cpp:11-18), and a transmit batch of
256 Ki messages with 0..1000-byte payloads wrapped in place and with the
headers apart (tcp_over_ip.cpp:69-88) — each call repeated so the later ones
run from the cached plan, the two sides interleaved as a tick does, against
the oracle."""
import numpy as np
import pytest

from helpers import pack_contiguous
from test_gpu_parity import _t, _u16

pytestmark = pytest.mark.gpu

N = 1 << 18


def _rx(rng):
    lens = np.where(rng.random(N) < 0.5, 40, 1500).astype(np.uint64)
    off = np.zeros(N + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    s = off[:-1].astype(np.int64)
    buf[s], buf[s + 1], buf[s + 2], buf[s + 3] = 0x45, 0, (lens >> 8).astype(np.uint8), (lens & 255).astype(np.uint8)
    buf[s + 6], buf[s + 7], buf[s + 8], buf[s + 9], buf[s + 32] = 0x40, 0, 64, 6, 0x50
    return buf, off


def _msgs(rng, n):
    from tcpip_network_protocol_stack_amd.engine import TCP_MSG_DTYPE

    m = np.zeros(n, dtype=TCP_MSG_DTYPE)
    for f, hi in (("src", 2**32), ("dst", 2**32), ("seqno", 2**32), ("ackno", 2**32), ("src_port", 2**16),
                  ("dst_port", 2**16), ("window", 2**16), ("id", 2**16)):
        m[f] = rng.integers(0, hi, n, dtype=np.uint64)
    m["flags"], m["ttl"] = 0x10, 128
    return m


def test_stack_tick_shapes_bit_exact(engine, orc):
    import torch

    from test_gpu_wrap import _oracle_wire

    rng = np.random.default_rng(0x57AC)
    buf, off = _rx(rng)
    orc.ipv4_tcp_batch(buf, N, 2, offsets=off)  # valid checksums ...
    s = off[:-1].astype(np.int64)
    buf[s[::10] + 25] ^= 0x04  # ... except every tenth datagram's TCP bytes
    want_v = orc.ipv4_tcp_batch(buf.copy(), N, 1, offsets=off)
    want_c = orc.ipv4_tcp_batch(buf.copy(), N, 0, offsets=off)
    assert 0 < int((want_v[2] == 0x0F).sum()) < N
    d, do = _t(buf), _t(off)
    # transmit side: 0..1000-byte payloads behind 40 bytes of room, and the same payloads alone
    pl = rng.integers(0, 1001, N)
    pays = [rng.integers(0, 256, int(x), dtype=np.uint8).tobytes() for x in pl]
    m = _msgs(rng, N)
    tb, toff = pack_contiguous([b"\0" * 40 + p for p in pays], 0)
    pb, poff = pack_contiguous(pays, 0)
    dm = torch.from_numpy(m.view(np.uint8).copy()).cuda()
    dp, dpo = _t(pb), _t(poff)
    kinds = []
    hd_first = None
    for call in range(3):
        ip, tcp, st = engine.ipv4_tcp_batch(d, 1, offsets=do)
        kinds.append(("verify", engine.dispatch_info()["kernel"]))
        assert (_u16(ip) == want_v[0]).all() and (_u16(tcp) == want_v[1]).all(), call
        assert (st.cpu().numpy() == want_v[2]).all(), call
        dt = _t(tb)
        engine.tcp_wrap_batch(dt, dm, n=N, offsets=_t(toff))
        kinds.append(("wrap", engine.dispatch_info()["kernel"]))
        ip, tcp, st = engine.ipv4_tcp_batch(d, 0, offsets=do)
        assert (_u16(ip) == want_c[0]).all() and (_u16(tcp) == want_c[1]).all(), call
        hd = torch.empty(N * 40, dtype=torch.uint8, device="cuda")
        engine.tcp_wrap_headers(dp, dm, hd, n=N, offsets=dpo)
        kinds.append(("apart", engine.dispatch_info()["kernel"]))
        h = hd.cpu().numpy().reshape(N, 40)
        w = dt.cpu().numpy()
        # in place and apart: the same 40 header bytes for every datagram, payloads untouched
        heads = w[toff[:-1].astype(np.int64)[:, None] + np.arange(40)]
        assert (heads == h).all(), call
        assert (dp.cpu().numpy() == pb).all()
        if hd_first is None:
            hd_first = h.copy()
        assert (h == hd_first).all(), call
    # ... and those are the reference's wire bytes (a sample through the oracle's wrap)
    idx = np.concatenate([np.arange(64), rng.choice(N, 3000, replace=False), np.arange(N - 64, N)])
    want_w = _oracle_wire(orc, [b"\0" * 40 + pays[i] for i in idx], m[idx])
    for k, i in enumerate(idx):
        got = w[int(toff[i]):int(toff[i + 1])].tobytes()
        assert got == want_w[k], i
    assert kinds[-3:] == [("verify", "ipv4_twoclass"), ("wrap", kinds[-2][1]), ("apart", "tile")], kinds
