#!/usr/bin/env python3
"""Dev measurement: the two-class launches (checksum and fused VERIFY) on the
receive mix (half 40-byte ACKs, half 1500-byte datagrams, valid headers,
packed offsets) with the blocks resident per CU capped by dynamic LDS
(ICSUM_FORCE twoclass_lds: bytes per block on top of the kernel's own) and
with 8 / 16 / 32 datagrams per wave (twoclass=N), at 256 Ki and 1 M
datagrams.  Two copies rotate; HIP events around 20 back-to-back calls,
median of 5 rounds."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _force import engine  # noqa: E402
from ab_stack import R, rx_batch, timed  # noqa: E402

import torch  # noqa: E402

PEAK = 8.0e12


def main():
    sizes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1 << 18, 1 << 20]
    pads = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 8192, 16384, 24576, 32768, 49152]
    auto = engine()
    engs = {f"lds{p}": (engine(twoclass_lds=p) if p else auto) for p in pads}
    engs.update({f"spw{w}": engine(twoclass=w) for w in (8, 16, 32)})
    engs.update({f"spw8_lds{p}": engine(twoclass=8, twoclass_lds=p) for p in (16384, 32768)})
    for n in sizes:
        rx = [rx_batch(auto, n, 11 + r) for r in range(R)]
        nb = rx[0][2]
        ip = torch.empty(n, dtype=torch.int16, device="cuda")
        tcp = torch.empty(n, dtype=torch.int16, device="cuda")
        st = torch.empty(n, dtype=torch.uint8, device="cuda")
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        for p, e in engs.items():
            t = timed(lambda i, e=e: e.ipv4_tcp_batch(rx[i % R][0], 1, n=n, offsets=rx[i % R][1], ip_ck=ip,
                                                      tcp_ck=tcp, status=st))
            assert (st.cpu().numpy() == 0x0F).all(), p
            k = e.dispatch_info()["kernel"]
            print(json.dumps({"row": f"verify_{n}", "lib": p, "bytes": nb, "us": round(t * 1e6, 2),
                              "frac": round(nb / t / PEAK, 4), "kernel": k}), flush=True)
            t = timed(lambda i, e=e: e.checksum_batch(rx[i % R][0], n=n, offsets=rx[i % R][1], out=out))
            k = e.dispatch_info()["kernel"]
            print(json.dumps({"row": f"checksum_{n}", "lib": p, "bytes": nb, "us": round(t * 1e6, 2),
                              "frac": round(nb / t / PEAK, 4), "kernel": k}), flush=True)
        del rx


if __name__ == "__main__":
    main()
