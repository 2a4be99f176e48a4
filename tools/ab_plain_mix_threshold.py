#!/usr/bin/env python3
"""Dev measurement: the plain checksum (AUTO, plan cached) against the forced
two-class launch (ICSUM_FORCE twoclass=16) on raw-datagram receive mixes at
low ACK shares — where the short-mix threshold (ics_ctx::kShortMix16) sits."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from _force import engine  # noqa: E402
from ab_ipv4_mix import batch, timed  # noqa: E402
from tcpip_network_protocol_stack_amd.engine import Engine  # noqa: E402


def main():
    shares = [float(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0.125, 0.1875, 0.25, 0.3125]
    auto, two = Engine(0), engine(twoclass=16)
    n = 1 << 20
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    for af in shares:
        d, doff, nbytes = batch(auto, n, af, 7)
        ta = timed(lambda: auto.checksum_batch(d, offsets=doff, out=out))
        ka = auto.dispatch_info()["kernel"]
        tt = timed(lambda: two.checksum_batch(d, offsets=doff, out=out))
        print(json.dumps({"ack_share": af, "bytes": nbytes, "auto_us": round(ta * 1e6, 2), "auto_kernel": ka,
                          "twoclass16_us": round(tt * 1e6, 2)}), flush=True)
        del d


if __name__ == "__main__":
    main()
