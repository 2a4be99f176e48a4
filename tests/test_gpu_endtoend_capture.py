"""GPU: the engine on the datagrams the UNMODIFIED reference stack put on the
wire in BASELINE config 1 (tests/golden/endtoend_capture.npz, made by
oracle/make_endtoend_capture.py from the reference's own apps/endtoend; the
CPU side is tests/test_endtoend_capture.py).  The reference wrote every
checksum on these bytes and accepted every datagram, so the engine must:
verify all of them (ICS_ST_ACCEPT, TCP value() 0), recompute exactly the
checksums on the wire, rebuild the wire from zeroed checksum fields (PATCH),
and forward them as the oracle does (router TTL step) — read where a receive
arena of Ethernet frames holds them (each datagram 14 bytes into its frame,
unaligned), from device memory, from host memory (the per-tick zero-copy
path) and as two batches in one multi-batch call (the two directions)."""
import numpy as np
import pytest

from helpers import endtoend_capture, ip_packed, pack_contiguous

pytestmark = pytest.mark.gpu


def _in_frames():
    """(frame buffer, frame offsets, direction, IPv4 starts, IPv4 ends)."""
    return endtoend_capture()


def _wire_checksums(data, off):
    n = len(off) - 1
    ip = np.empty(n, dtype=np.uint16)
    tcp = np.empty(n, dtype=np.uint16)
    for i in range(n):
        s = int(off[i])
        t = 4 * (int(data[s]) & 0x0F)
        ip[i] = int(data[s + 10]) << 8 | int(data[s + 11])
        tcp[i] = int(data[s + t + 16]) << 8 | int(data[s + t + 17])
    return ip, tcp


@pytest.mark.parametrize("lead", [0, 14])
def test_capture_device_every_mode(engine, orc, lead):
    import torch

    buf, _, _, starts, ends = _in_frames()
    data, off = ip_packed(buf, starts, ends, lead)
    n = len(off) - 1
    want_ip, want_tcp = _wire_checksums(data, off)
    d = torch.from_numpy(data.copy()).cuda()
    doff = torch.from_numpy(off.view(np.int64).copy()).cuda()
    ip, tcp, st = engine.ipv4_tcp_batch(d, 1, n=n, offsets=doff)
    assert (st.cpu().numpy() == 0x0F).all() and (tcp.cpu().numpy() == 0).all()
    ip, tcp, st = engine.ipv4_tcp_batch(d, 0, n=n, offsets=doff)
    assert (ip.cpu().numpy().view(np.uint16) == want_ip).all()
    assert (tcp.cpu().numpy().view(np.uint16) == want_tcp).all()
    zeroed = data.copy()
    for i in range(n):
        s = int(off[i])
        t = 4 * (int(zeroed[s]) & 0x0F)
        zeroed[s + 10:s + 12] = 0
        zeroed[s + t + 16:s + t + 18] = 0
    dz = torch.from_numpy(zeroed).cuda()
    engine.ipv4_tcp_batch(dz, 2, n=n, offsets=doff)
    torch.cuda.synchronize()
    assert (dz.cpu().numpy() == data).all()
    # the TCP checksum alone: InternetChecksum{pseudo}.add(segment).value() == 0
    # (tcp_segment.cpp:11-18), through the plain checksum entry point
    seg_off = off.copy()
    seg_off[:-1] += 20  # every captured header is 20 bytes
    segs = [data[int(seg_off[i]):int(off[i + 1])].tobytes() for i in range(n)]
    sb, so = pack_contiguous(segs, lead)
    pseudo = np.empty(n, dtype=np.uint32)  # IPv4Header::pseudo_checksum (ipv4_header.cpp:103-110)
    for i in range(n):
        h = data[int(off[i]):int(off[i]) + 20]
        src, dst = int.from_bytes(h[12:16].tobytes(), "big"), int.from_bytes(h[16:20].tobytes(), "big")
        plen = (int.from_bytes(h[2:4].tobytes(), "big") - 20) & 0xFFFF
        pseudo[i] = (src >> 16) + (src & 0xFFFF) + (dst >> 16) + (dst & 0xFFFF) + 6 + plen
    v = engine.checksum_batch(torch.from_numpy(sb).cuda(), n=n, offsets=torch.from_numpy(so.view(np.int64)).cuda(),
                              init=torch.from_numpy(pseudo.view(np.int32)).cuda())
    assert (v.cpu().numpy() == 0).all()


def test_capture_router_step(engine, orc):
    import torch

    buf, _, _, starts, ends = _in_frames()
    data, off = ip_packed(buf, starts, ends, 14)
    n = len(off) - 1
    d = torch.from_numpy(data.copy()).cuda()
    st = engine.router_ttl_batch(d, n=n, offsets=torch.from_numpy(off.view(np.int64).copy()).cuda())
    got = d.cpu().numpy()
    assert (st.cpu().numpy() == 1).all()
    for i in range(n):
        s, e = int(off[i]), int(off[i + 1])
        ost, fwd = orc.router_ttl(data[s:e].tobytes())
        assert ost == 1 and got[s:e].tobytes() == fwd, i


@pytest.mark.parametrize("pinned", [False, True])
def test_capture_host_path(engine, orc, pinned):
    import torch

    buf, _, _, starts, ends = _in_frames()
    data, off = ip_packed(buf, starts, ends, 14)
    n = len(off) - 1
    h = torch.empty(data.size, dtype=torch.uint8, pin_memory=pinned).numpy()
    h[:] = data
    ip, tcp, st = engine.ipv4_tcp_batch_host(h, n, 1, offsets=off)
    assert (st == 0x0F).all() and (tcp == 0).all()
    ip, tcp, st = engine.ipv4_tcp_batch_host(h, n, 0, offsets=off)
    want_ip, want_tcp = _wire_checksums(data, off)
    assert (ip == want_ip).all() and (tcp == want_tcp).all()
    # one tick per datagram, as the reference's TUN read hands them over
    for i in range(0, n, 17):
        one = data[int(off[i]):int(off[i + 1])].copy()
        _, t1, s1 = engine.ipv4_tcp_batch_host(one, 1, 1, offsets=np.array([0, one.size], dtype=np.uint64))
        assert s1[0] == 0x0F and t1[0] == 0, i


def test_capture_two_directions_one_multibatch_call(engine):
    import torch

    buf, off_f, direction, starts, ends = _in_frames()
    is_ip = [i for i in range(len(off_f) - 1) if buf[off_f[i] + 12] == 0x08 and buf[off_f[i] + 13] == 0]
    dirs = direction[is_ip]
    batches, keep = [], []
    for dv in (0, 1):
        sel = dirs == dv
        data, off = ip_packed(buf, starts[sel], ends[sel], 14)
        n = len(off) - 1
        d = torch.from_numpy(data).cuda()
        doff = torch.from_numpy(off.view(np.int64).copy()).cuda()
        st = torch.empty(n, dtype=torch.uint8, device="cuda")
        tcp = torch.empty(n, dtype=torch.int16, device="cuda")
        keep += [d, doff]
        batches.append(dict(dgrams=d, offsets=doff, n=n, status=st, tcp_ck=tcp))
    engine.ipv4_tcp_batchv(batches, 1)
    torch.cuda.synchronize()
    for b in batches:
        assert (b["status"].cpu().numpy() == 0x0F).all() and (b["tcp_ck"].cpu().numpy() == 0).all()
