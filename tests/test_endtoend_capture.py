"""CPU: the oracle on the datagrams the UNMODIFIED reference stack put on
the wire in BASELINE config 1 (tests/golden/endtoend_capture.npz, made by
oracle/make_endtoend_capture.py from the reference's own apps/endtoend):
every TCP checksum was written by the reference's
TCPSegment::compute_checksum (util/tcp_over_ip/tcp_over_ip.cpp:83) and every
header checksum rewritten by its router after the TTL decrement
(src/router/router.cpp:43-50), and the stack accepted them all.  The oracle
must verify every one, recompute exactly the checksums on the wire, and
rebuild the wire bytes from datagrams whose checksum fields were zeroed."""
import numpy as np

from helpers import endtoend_capture, ip_packed


def test_capture_shape():
    buf, off, direction, starts, ends = endtoend_capture()
    n = len(off) - 1
    assert n > 200 and len(starts) >= n - 4  # IPv4 frames, plus a few ARP
    assert set(direction.tolist()) == {0, 1}
    assert (ends - starts >= 40).all()  # every IPv4 frame carries a TCP segment


def test_oracle_verifies_and_reproduces_reference_wire(orc):
    buf, _, _, starts, ends = endtoend_capture()
    data, off = ip_packed(buf, starts, ends, lead=3)
    n = len(off) - 1
    ip, tcp, st = orc.ipv4_tcp_batch(data.copy(), n, 1, offsets=off)
    assert (st == 0x0F).all() and (tcp == 0).all()
    ipc, tcpc, st = orc.ipv4_tcp_batch(data.copy(), n, 0, offsets=off)
    for i in range(n):
        d = data[int(off[i]):int(off[i + 1])]
        t = 4 * (int(d[0]) & 0x0F)
        assert ipc[i] == (int(d[10]) << 8 | int(d[11])), i
        assert tcpc[i] == (int(d[t + 16]) << 8 | int(d[t + 17])), i
    zeroed = data.copy()
    for i in range(n):
        s = int(off[i])
        t = 4 * (int(zeroed[s]) & 0x0F)
        zeroed[s + 10:s + 12] = 0
        zeroed[s + t + 16:s + t + 18] = 0
    orc.ipv4_tcp_batch(zeroed, n, 2, offsets=off)
    assert (zeroed == data).all()


def test_oracle_router_step_on_captured_datagrams(orc):
    buf, _, _, starts, ends = endtoend_capture()
    for s, e in zip(starts, ends):
        d = buf[int(s):int(e)].tobytes()
        st, fwd = orc.router_ttl(d)
        assert st == 1 and fwd[8] == d[8] - 1
        assert orc.ipv4_tcp(fwd, 1)[2] == 0x0F
