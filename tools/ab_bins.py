#!/usr/bin/env python3
"""Dev tool: where a split-plan binned batch loses time.  One bin's worth of
segments (1 M x 1460-1463 B, or 1 M x 40-43 B) through the binned dispatch
(split plan forced), through the single long-segment launch, and through a
single launch with the bin's own geometry (one lane group per segment, no
list, no grid stride); interleaved in one process.  (Round 1 also ran the
bin's geometry on a capped grid, a knob since removed: profiles/r1_ab_bins*.)

    python tools/ab_bins.py [--rounds 5]
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
    "binned_split": {"bin": 1, "bin_plan": 1},
    "single_64x8": {"bin": 0},
    "single_16x8m3": {"bin": 0, **geometry(16, 8, 3)},
    "single_4x2s2": {"bin": 0, **geometry(4, 2, 2, segs=2)},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    engs = {k: engine(**v) for k, v in VARIANTS.items()}
    st = torch.cuda.current_stream()
    rng = np.random.default_rng(0x1460)
    n = 1 << 20
    for kind, base in (("mss_1460", 1460), ("ack_40", 40)):
        lens = base + rng.integers(0, 4, n)
        off = np.zeros(n + 1, dtype=np.int64)
        off[1:] = np.cumsum(lens)
        nbytes = int(off[-1])
        e0 = engs["single_64x8"]
        d = e0.fill_bytes(torch.empty(nbytes + 16, dtype=torch.uint8, device=dev), 0x1460)
        doff = torch.from_numpy(off).to(dev)
        ref = e0.checksum_batch(d, offsets=doff)
        torch.cuda.synchronize()
        names = [k for k in engs if not (kind == "mss_1460" and k == "single_4x2s2")]
        times = {k: [] for k in names}
        for r in range(args.rounds):
            for k in names if r % 2 == 0 else names[::-1]:
                out = torch.empty_like(ref)
                engs[k].checksum_batch(d, offsets=doff, out=out)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(args.iters):
                    engs[k].checksum_batch(d, offsets=doff, out=out)
                b.record(st)
                torch.cuda.synchronize()
                assert torch.equal(out, ref), (kind, k)
                times[k].append(a.elapsed_time(b) * 1e3 / args.iters)
        for k, ts in times.items():
            med = statistics.median(ts)
            print(json.dumps({"workload": kind, "bytes": nbytes, "variant": k, "med_us": round(med, 2),
                              "GB_s": round(nbytes / med / 1e3, 1)}), flush=True)
        del d, doff


if __name__ == "__main__":
    main()
