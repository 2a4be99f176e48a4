#!/usr/bin/env python3
"""Dev tool: interleaved in-process A/B of the binned dispatch's last-bin
launch, each value an ICSUM_FORCE key: its grid cap (last_bin_blocks; 0 = one
lane group per segment of the batch), its lanes per segment (--var
last_bin_lps --caps 64,32) or the plan (--var bin_plan --caps=0,1,2,3,-1; -1 =
decided on the device; --var bin --caps=-1,1 compares the plan cache with
binning on every call).  Workloads: BASELINE config 4 (1 M mixed 64 B-64 KiB,
whole-batch plan), the 2 M bimodal 40 B / 1460 B batch (split plan, empty last
bin) and 2 M segments of 4-6 KiB (whole-batch plan with > 1 M segments).

    python tools/ab_lastbin.py [--caps 0,262144,131072] [--rounds 5]
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

from tcpip_network_protocol_stack_amd.engine import mixed_offsets  # noqa: E402
from _force import engine as forced  # noqa: E402


VAR = "last_bin_blocks"


def engine(cap):
    return forced(**{VAR: cap})


def batch(kind, dev, eng):
    if kind == "config4":
        off = mixed_offsets(1 << 20, 0x10710004).astype(np.int64)
    elif kind in ("mss", "ack"):
        rng = np.random.default_rng(0x1460)
        lens = (1460 if kind == "mss" else 40) + rng.integers(0, 4, 1 << 20)
        off = np.zeros(lens.size + 1, dtype=np.int64)
        off[1:] = np.cumsum(lens)
    else:
        rng = np.random.default_rng(0x10710006)
        n = 2 << 20
        lens = (np.where(rng.random(n) < 0.5, 40, 1460) + rng.integers(0, 4, n) if kind == "bimodal"
                else rng.integers(4096, 6144, n))
        off = np.zeros(n + 1, dtype=np.int64)
        off[1:] = np.cumsum(lens)
    d = eng.fill_bytes(torch.empty(int(off[-1]) + 16, dtype=torch.uint8, device=dev), 0x10710004)
    return d, torch.from_numpy(off).to(dev), off.size - 1, int(off[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--caps", default="0,262144,131072")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--var", default="last_bin_blocks", help="ICSUM_FORCE key")
    ap.add_argument("--workloads", default="config4,bimodal,long2m", help="config4,bimodal,long2m,mss,ack")
    args = ap.parse_args()
    global VAR
    VAR = args.var
    dev = torch.device("cuda", 0)
    caps = [int(c) for c in args.caps.split(",")]
    engs = {c: engine(c) for c in caps}
    st = torch.cuda.current_stream()
    for kind in args.workloads.split(","):
        d, off, n, nbytes = batch(kind, dev, engs[caps[0]])
        out = {c: torch.empty(n, dtype=torch.int16, device=dev) for c in caps}
        for c in caps:
            engs[c].checksum_batch(d, offsets=off, out=out[c])
        torch.cuda.synchronize()
        for c in caps[1:]:
            assert torch.equal(out[c], out[caps[0]]), (kind, c)
        times = {c: [] for c in caps}
        for r in range(args.rounds):
            for c in caps if r % 2 == 0 else caps[::-1]:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(args.iters):
                    engs[c].checksum_batch(d, offsets=off, out=out[c])
                b.record(st)
                torch.cuda.synchronize()
                times[c].append(a.elapsed_time(b) * 1e3 / args.iters)
        for c, ts in times.items():
            med = statistics.median(ts)
            print(json.dumps({"workload": kind, "segments": n, "bytes": nbytes, VAR: c,
                              "med_us": round(med, 2), "min_us": round(min(ts), 2),
                              "GB_s": round(nbytes / med / 1e3, 1)}), flush=True)
        del d, off
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
