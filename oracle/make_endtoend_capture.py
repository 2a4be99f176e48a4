#!/usr/bin/env python3
"""Fixture generator (test infrastructure): the frames the UNMODIFIED reference
stack exchanges in BASELINE config 1, captured on the relay.

Runs the reference's own apps/endtoend (built in place from /root/reference
by `make -C tcpip_network_protocol_stack_amd/csrc/host/integration reference`
into oracle/_ref/apps/endtoend — no drop-in code in it) for a 128 KiB
client -> server transfer over tools/endtoend_run.py's UDP bounce relay, and
saves every relayed frame: serialized EthernetFrames between the two routers
(/root/reference/apps/endtoend.cpp:118-124), i.e. IPv4 datagrams whose TCP
checksum the reference's TCPSegment::compute_checksum wrote
(util/tcp_over_ip/tcp_over_ip.cpp:83) and whose header checksum its router
rewrote after the TTL decrement (src/router/router.cpp:43-50), plus ARP.

    python oracle/make_endtoend_capture.py  ->  tests/golden/endtoend_capture.npz

The stack accepted every one of these datagrams; the tests check the oracle
and the engine against the checksums on the wire."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFBIN = os.path.join(ROOT, "oracle", "_ref", "apps", "endtoend")
INTEG = os.path.join(ROOT, "tcpip_network_protocol_stack_amd", "csrc", "host", "integration")
OUT = os.path.join(ROOT, "tests", "golden", "endtoend_capture.npz")


def main():
    subprocess.check_call(["make", "-s", "-j", "8", "-C", INTEG, "reference"])
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "endtoend_run.py"), REFBIN, "--bytes",
                        str(128 << 10), "--timeout", "90", "--capture", OUT], capture_output=True, text=True,
                       timeout=240)
    line = json.loads(r.stdout.strip().splitlines()[-1])
    if r.returncode != 0 or not line["ok"]:
        sys.exit(f"endtoend failed: {line} {r.stderr[-2000:]}")
    print(json.dumps(line))


if __name__ == "__main__":
    main()
