#!/usr/bin/env python3
"""Dev tool: interleaved A/B of the XCD-aware block order (ICSUM_FORCE
xcd_remap) on fixed-stride workloads.  The toggle is process-wide and set when
an engine is created, so each round re-creates the engine with the variant.

    python tools/ab_xcd.py [--workloads ns,s576,jumbo] [--rounds 7] [--iters 40]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from _force import engine  # noqa: E402

WL = {"ns": (1 << 20, 1500), "s576": (1 << 21, 576), "jumbo": (1 << 19, 9000), "s3000": (1 << 19, 3000),
      "jumbo1m": (1 << 20, 9000), "jumbo8m": (8 << 20, 9000)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="ns,s576,jumbo")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--variants", default="0,1", help="xcd_remap values: log2 of the XCD run length in blocks, 0 = hardware order")
    args = ap.parse_args()
    st = torch.cuda.current_stream()
    for wl in args.workloads.split(","):
        n, L = WL[wl]
        seed = 0x10710000
        base = engine(xcd_remap=1)
        data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        base.fill_bytes(data, seed)
        init = base.pseudo_inits(n, seed, seg_len=L)
        ref = base.checksum_batch(data, n=n, stride=L, seg_len=L, init=init)
        torch.cuda.synchronize()
        base.close()
        variants = [int(v) for v in args.variants.split(",")]
        times = {v: [] for v in variants}
        # settle: ~200 ms of launches before the first timed round
        eng = engine(xcd_remap=0)
        out = torch.empty_like(ref)
        for _ in range(max(8, int(0.2 / (n * L / 7e12)))):
            eng.checksum_batch(data, n=n, stride=L, seg_len=L, init=init, out=out)
        torch.cuda.synchronize()
        eng.close()
        for r in range(args.rounds):
            for v in variants if r % 2 == 0 else variants[::-1]:
                eng = engine(xcd_remap=v)
                eng.checksum_batch(data, n=n, stride=L, seg_len=L, init=init, out=out)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(args.iters):
                    eng.checksum_batch(data, n=n, stride=L, seg_len=L, init=init, out=out)
                b.record(st)
                torch.cuda.synchronize()
                times[v].append(a.elapsed_time(b) / args.iters / 1e3)
                assert torch.equal(out, ref), f"remap={v} mismatch"
                eng.close()
        for v, ts in times.items():
            med = statistics.median(ts)
            print(json.dumps({"workload": wl, "xcd_remap": v, "med_us": round(med * 1e6, 2),
                              "med_GBs": round(n * L / med / 1e9, 1), "best_GBs": round(n * L / min(ts) / 1e9, 1)}),
                  flush=True)
        del data


if __name__ == "__main__":
    main()
