#!/usr/bin/env python3
"""Dev tool: interleaved in-process A/B of kernel geometries (LPS, UNROLL,
MODE, SEGS through ICSUM_FORCE; the load policy follows the geometry table)
on the BASELINE workloads (cdna_hip_programming.md §5.4 rule 24).

    python tools/sweep_geometry.py [--workloads ns,tcp64,jumbo,mixed] [--rounds 5]
Prints one JSON line per (workload, variant) with median/min kernel GB/s.
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

from tcpip_network_protocol_stack_amd.engine import Engine, mixed_offsets  # noqa: E402
from _force import engine, geometry  # noqa: E402

WL = {"ns": (1 << 20, 1500), "tcp64": (1 << 20, 64), "jumbo": (1 << 20, 9000), "mixed": (1 << 20, None),
      "s128": (1 << 20, 128), "s256": (1 << 20, 256), "s576": (1 << 20, 576), "s3000": (1 << 19, 3000),
      "s600": (1 << 20, 600), "s800": (1 << 20, 800), "s1000": (1 << 20, 1000), "s1040": (1 << 20, 1040),
      "s1200": (1 << 20, 1200), "s1460": (1 << 20, 1460), "s2000": (1 << 20, 2000),
      "s2500": (1 << 19, 2500), "s4096": (1 << 19, 4096), "s6000": (1 << 18, 6000),
      "s1400": (1 << 20, 1400), "s1536": (1 << 20, 1536), "s1600": (1 << 20, 1600), "s1800": (1 << 20, 1800)}


def make_engine(lps, unroll, mode, segs):
    return engine(**geometry(lps, unroll, mode, segs=segs if segs > 1 else None))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="ns,tcp64,jumbo,mixed")
    ap.add_argument("--variants", default="")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    # LPSxUNROLL[xMODE[xSEGS]]
    def parse_variant(v):
        parts = [int(x) for x in v.split("x")]
        return tuple(parts + [3, 1][len(parts) - 2:])[:4]  # defaults: MODE 3 (line grid), SEGS 1

    variants = [parse_variant(v) for v in args.variants.split(",") if v] or [
        (16, 8, 3, 1), (32, 8, 3, 1), (64, 8, 3, 1), (4, 2, 2, 2)]
    base = Engine(0)
    for wl in args.workloads.split(","):
        n, L = WL[wl]
        seed = 0x10710000
        if L is None:
            off = mixed_offsets(n, 0x10710004)
            total = int(off[-1])
            doff = torch.from_numpy(off.view(np.int64)).cuda()
        else:
            total, doff = n * L, None
        data = torch.empty(total, dtype=torch.uint8, device="cuda")
        base.fill_bytes(data, seed)
        init = base.pseudo_inits(n, seed, offsets=doff, seg_len=L or 0)
        ref = base.checksum_batch(data, n=n, offsets=doff, stride=L or 0, seg_len=L or 0, init=init)
        torch.cuda.synchronize()
        engines = {}
        for lps, u, mode, segs in variants:
            engines[(lps, u, mode, segs)] = make_engine(lps, u, mode, segs)
        times = {k: [] for k in engines}
        st = torch.cuda.current_stream()
        for r in range(args.rounds):
            for k, eng in engines.items():
                out = eng.checksum_batch(data, n=n, offsets=doff, stride=L or 0, seg_len=L or 0, init=init)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(args.iters):
                    eng.checksum_batch(data, n=n, offsets=doff, stride=L or 0, seg_len=L or 0, init=init, out=out)
                b.record(st)
                torch.cuda.synchronize()
                times[k].append(a.elapsed_time(b) / args.iters / 1e3)
                if r == 0:
                    assert torch.equal(out, ref), f"variant {k} mismatch"
        for k, ts in times.items():
            med = statistics.median(ts)
            print(json.dumps({"workload": wl, "lps": k[0], "unroll": k[1], "mode": k[2], "segs": k[3],
                              "med_us": round(med * 1e6, 1), "med_GBs": round(total / med / 1e9, 1),
                              "best_GBs": round(total / min(ts) / 1e9, 1)}), flush=True)
        for e in engines.values():
            e.close()
        del data


if __name__ == "__main__":
    main()
