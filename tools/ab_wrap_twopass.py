#!/usr/bin/env python3
"""Dev A/B: the device wrap as two passes (payload sums, then a header launch;
ICSUM_FORCE wrap_passes=2) vs the one-pass kernel that stores the headers inside the
payload stream (wrap_passes=1), beside the plain checksum of the same
payloads (the default picks two passes for headers apart, one in place).
1 M x 1000-byte payloads / 1040-byte datagrams, interleaved rounds in one
process; also 64 Ki x 1500 B (config 2's shape)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tcpip_network_protocol_stack_amd.engine import TCP_MSG_DTYPE  # noqa: E402
from _force import engine  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    two = engine(wrap_passes=2)
    one = engine(wrap_passes=1)
    for n, L in ((1 << 20, 1040), (1 << 16, 1500)):
        P, R = L - 40, max(3, (600 << 20) // (n * L) + 1)
        rng = np.random.default_rng(6)
        m = np.zeros(n, dtype=TCP_MSG_DTYPE)
        for f in ("src", "dst", "seqno", "ackno"):
            m[f] = rng.integers(0, 2**32, n, dtype=np.uint64)
        m["flags"], m["ttl"] = 0x10, 128
        dm = torch.from_numpy(m.view(np.uint8).copy()).to(dev)
        ps = [two.fill_bytes(torch.empty(n * P, dtype=torch.uint8, device=dev), 0x1071, pos0=r * n * P)
              for r in range(R)]
        ds = [two.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), 0x1072, pos0=r * n * L)
              for r in range(R)]
        hd = torch.empty(n * 40, dtype=torch.uint8, device=dev)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        cases = {"plain": lambda i: two.checksum_batch(ps[i % R], n=n, stride=P, seg_len=P, out=out)}
        for nm, e in (("two_pass", two), ("fused", one)):
            cases[f"apart_{nm}"] = (lambda e: lambda i: e.tcp_wrap_headers(ps[i % R], dm, hd, n=n, stride=P,
                                                                            payload_len=P))(e)
            cases[f"in_place_{nm}"] = (lambda e: lambda i: e.tcp_wrap_batch(ds[i % R], dm, n=n, stride=L,
                                                                             dgram_len=L))(e)
        res = {k: [] for k in cases}
        st = torch.cuda.current_stream()
        for rnd in range(5):
            for k, fn in cases.items():
                t0 = time.perf_counter()
                while time.perf_counter() - t0 < 0.04:
                    for i in range(4):
                        fn(i)
                    torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for i in range(20):
                    fn(i)
                b.record(st)
                torch.cuda.synchronize()
                res[k].append(a.elapsed_time(b) * 1e3 / 20)
        print(json.dumps({"n": n, "dgram_len": L, **{k: round(float(np.median(v)), 2) for k, v in res.items()}}),
              flush=True)
        del ps, ds


if __name__ == "__main__":
    main()
