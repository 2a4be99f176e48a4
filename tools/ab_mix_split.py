#!/usr/bin/env python3
"""Dev measurement: a received ACK/MTU mix (raw datagrams back to back,
valid IPv4 headers) VERIFYed in one call (the default dispatch: the two-class
launch from 5/16 ACKs up) against the same datagrams repacked by class into
an ACK-only and an MTU-only batch, each VERIFYed in its own call — the
"classes apart" floor the one-call launch is measured against.
Argument: datagram count (default 1 M), ACK shares (default 0.5)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ab_ipv4_mix import batch, timed  # noqa: E402
from tcpip_network_protocol_stack_amd.engine import Engine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    shares = [float(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0.5]
    eng = Engine(0)
    dev = torch.device("cuda", 0)
    for af in shares:
        d, doff, _ = batch(eng, n, af, 11)
        off = doff.cpu().numpy().view(np.uint64)
        lens = np.diff(off)
        host = d.cpu().numpy()
        outs = [torch.empty(n, dtype=t, device=dev) for t in (torch.int16, torch.int16, torch.uint8)]
        t_one = timed(lambda: eng.ipv4_tcp_batch(d, 1, n=n, offsets=doff, ip_ck=outs[0], tcp_ck=outs[1],
                                                 status=outs[2]))
        info = eng.dispatch_info()
        parts = {}
        for name, sel in (("acks", lens <= 64), ("mtu", lens > 64)):
            idx = np.nonzero(sel)[0]
            segs = [host[int(off[i]):int(off[i + 1])] for i in idx]
            po = np.zeros(len(idx) + 1, dtype=np.uint64)
            po[1:] = np.cumsum([s.size for s in segs])
            pd = torch.from_numpy(np.concatenate(segs + [np.zeros(16, np.uint8)])).to(dev)
            pdo = torch.from_numpy(po.view(np.int64)).to(dev)
            m = len(idx)
            t = timed(lambda: eng.ipv4_tcp_batch(pd, 1, n=m, offsets=pdo, ip_ck=outs[0], tcp_ck=outs[1],
                                                 status=outs[2]))
            parts[name] = (m, t, eng.dispatch_info()["kernel"])
        total = int(off[-1])
        print(json.dumps({"n": n, "ack_share": af, "bytes": total, "one_call_us": round(t_one * 1e6, 2),
                          "one_call_kernel": info["kernel"], "one_call_frac": round(total / t_one / 8e12, 4),
                          "apart_us": round((parts["acks"][1] + parts["mtu"][1]) * 1e6, 2),
                          "acks": [parts["acks"][0], round(parts["acks"][1] * 1e6, 2), parts["acks"][2]],
                          "mtu": [parts["mtu"][0], round(parts["mtu"][1] * 1e6, 2), parts["mtu"][2]]}), flush=True)


if __name__ == "__main__":
    main()
