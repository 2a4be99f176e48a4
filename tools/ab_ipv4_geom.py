#!/usr/bin/env python3
"""Dev A/B: lane-group geometry of the fused IPv4/TCP kernel on BASELINE
config 2 (64 Ki x 1500 B, 6 rotated copies), COMPUTE / VERIFY / PATCH,
engines with forced geometries (ICSUM_FORCE lps/unroll/mode) interleaved in one process."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from _force import engine, geometry  # noqa: E402


def main():
    variants = [v for v in (sys.argv[1] if len(sys.argv) > 1 else "16x8x3,32x4x3,16x6x3,32x3x3,16x5x3").split(",")]
    engs = {v: engine(**geometry(*map(int, v.split("x")))) for v in variants}
    dev = torch.device("cuda", 0)
    n, L, seed, R = 1 << 16, 1500, 0x10710002, 6
    base = engs[variants[0]]
    bufs = []
    for r in range(R):
        d = base.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L)
        base.ipv4_tcp_headers(d, n, L, L, seed, index0=r * n)
        base.ipv4_tcp_batch(d, 2, n=n, stride=L, dgram_len=L)
        bufs.append(d)
    ip = torch.empty(n, dtype=torch.int16, device=dev)
    tcp = torch.empty(n, dtype=torch.int16, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    res = {(v, m): [] for v in variants for m in (0, 1, 2)}
    for rnd in range(7):
        for v, e in engs.items():
            for m in (0, 1, 2):
                t0 = time.perf_counter()
                while time.perf_counter() - t0 < 0.03:
                    for i in range(8):
                        e.ipv4_tcp_batch(bufs[i % R], m, n=n, stride=L, dgram_len=L, ip_ck=ip, tcp_ck=tcp, status=st)
                    torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for i in range(60):
                    e.ipv4_tcp_batch(bufs[i % R], m, n=n, stride=L, dgram_len=L, ip_ck=ip, tcp_ck=tcp, status=st)
                b.record()
                torch.cuda.synchronize()
                res[(v, m)].append(a.elapsed_time(b) * 1e3 / 60)
    for (v, m), ts in res.items():
        print(json.dumps({"variant": v, "mode": ["compute", "verify", "patch"][m],
                          "med_us": round(statistics.median(ts), 2)}), flush=True)


if __name__ == "__main__":
    main()
