#!/usr/bin/env python3
"""Dev tool: lane geometry of the fused IPv4/TCP kernel on OFFSETS batches
(raw datagrams back to back, the DatagramBatch / TUN receive layout), where
the engine has no length hint.  Interleaved in one process, 6 rotated copies
so launches read HBM.  Workloads: 64 Ki x 1500 B (MTU) and 16 Ki x 9000 B
(jumbo) datagrams, VERIFY mode.

    python tools/ab_ipv4_offsets.py [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from _force import engine, geometry  # noqa: E402

VARIANTS = {
    "default": {},
    "16x8m3": geometry(16, 8, 3),
    "32x4m3": geometry(32, 4, 3),
    "64x8m3": geometry(64, 8, 3),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    engs = {k: engine(**v) for k, v in VARIANTS.items()}
    st = torch.cuda.current_stream()
    base = engs["default"]
    for n, L, seed in ((1 << 16, 1500, 0x10710002), (1 << 14, 9000, 0x10710005)):
        R = 6
        bufs = []
        for r in range(R):
            d = base.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L)
            base.ipv4_tcp_headers(d, n, L, L, seed, index0=r * n)
            base.ipv4_tcp_batch(d, 2, n=n, stride=L, dgram_len=L)  # valid checksums
            bufs.append(d)
        off = torch.from_numpy((np.arange(n + 1, dtype=np.int64) * L)).to(dev)
        ip = torch.empty(n, dtype=torch.int16, device=dev)
        tcp = torch.empty(n, dtype=torch.int16, device=dev)
        stt = torch.empty(n, dtype=torch.uint8, device=dev)
        times = {k: [] for k in engs}
        for r in range(args.rounds):
            for k in (list(engs) if r % 2 == 0 else list(engs)[::-1]):
                e = engs[k]
                e.ipv4_tcp_batch(bufs[0], 1, offsets=off, ip_ck=ip, tcp_ck=tcp, status=stt)
                torch.cuda.synchronize()
                assert bool((stt == 0x0F).all()), k
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for i in range(args.iters):
                    e.ipv4_tcp_batch(bufs[i % R], 1, offsets=off, ip_ck=ip, tcp_ck=tcp, status=stt)
                b.record(st)
                torch.cuda.synchronize()
                times[k].append(a.elapsed_time(b) * 1e3 / args.iters)
        for k, ts in times.items():
            med = statistics.median(ts)
            print(json.dumps({"datagrams": n, "len": L, "variant": k, "med_us": round(med, 2),
                              "GB_s": round(n * L / med / 1e3, 1)}), flush=True)
        del bufs


if __name__ == "__main__":
    main()
