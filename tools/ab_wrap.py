#!/usr/bin/env python3
"""Dev A/B: device-side wrap in one kernel (headers written in place) vs the
split variant (ICSUM_WRAP_SPLIT=1: compact headers, then an address-ordered
scatter launch), interleaved in one process on the same 1 M x 1040 B batch."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tcpip_network_protocol_stack_amd.engine import TCP_MSG_DTYPE, Engine  # noqa: E402


def main():
    engines = {"fused": Engine(0)}
    os.environ["ICSUM_WRAP_SPLIT"] = "1"
    engines["split"] = Engine(0)
    del os.environ["ICSUM_WRAP_SPLIT"]
    dev = torch.device("cuda", 0)
    for n, L in ((1 << 20, 1040), (1 << 16, 1500), (1 << 20, 200)):
        rng = np.random.default_rng(1)
        m = np.zeros(n, dtype=TCP_MSG_DTYPE)
        m["seqno"] = rng.integers(0, 2**32, n, dtype=np.uint64)
        m["flags"], m["ttl"] = 0x10, 128
        dm = torch.from_numpy(m.view(np.uint8).copy()).to(dev)
        R = max(2, (400 << 20) // (n * L) + 1)
        ds = [engines["fused"].fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), 0x1071, pos0=r * n * L)
              for r in range(R)]
        res = {k: [] for k in engines}
        for rnd in range(5):
            for k, e in engines.items():
                t0 = time.perf_counter()
                while time.perf_counter() - t0 < 0.05:
                    e.tcp_wrap_batch(ds[0], dm, n=n, stride=L, dgram_len=L)
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for i in range(20):
                    e.tcp_wrap_batch(ds[i % R], dm, n=n, stride=L, dgram_len=L)
                b.record()
                torch.cuda.synchronize()
                res[k].append(a.elapsed_time(b) * 1e3 / 20)
        print(json.dumps({"n": n, "L": L, **{k: round(float(np.median(v)), 2) for k, v in res.items()}}), flush=True)
        del ds


if __name__ == "__main__":
    main()
