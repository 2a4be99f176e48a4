#!/usr/bin/env python3
"""Dev tool: config 3 (1 M x 64 B with pseudo-header inits) through the dense
kernel — one batch per call, one 8 M-segment batch (the same bytes as eight
batches), and eight batches per ics_checksum_batchv call (round 3 also
measured 8 segments per lane group in flight and hardware block order for
the multi-batch dense class: within noise, profiles/r3_ab_batchv_config3*) — interleaved in one process, outputs of
every variant compared.  Prints one JSON line per variant: us per 1 M-segment
batch and the fraction of 8 TB/s of segment bytes.

    python tools/ab_batchv.py [--rounds 5] [--iters 20]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from tcpip_network_protocol_stack_amd.engine import Engine  # noqa: E402


def engine(**force):
    if force:
        os.environ["ICSUM_FORCE"] = ",".join(f"{k}={v}" for k, v in force.items())
    try:
        return Engine(0)
    finally:
        os.environ.pop("ICSUM_FORCE", None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, L, seed, K = 1 << 20, 64, 0x10710003, 8
    e4, s8 = engine(), engine(dense_segs=8)
    big = e4.fill_bytes(torch.empty(2 * K * n * L, dtype=torch.uint8, device=dev), seed)
    binit = e4.pseudo_inits(2 * K * n, seed, seg_len=L)
    ds = [big[r * n * L:(r + 1) * n * L] for r in range(2 * K)]
    inits = [binit[r * n:(r + 1) * n] for r in range(2 * K)]
    outs = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(K)]
    bout = torch.empty(K * n, dtype=torch.int16, device=dev)
    sets = [[dict(data=ds[s * K + j], n=n, stride=L, seg_len=L, init=inits[s * K + j], out=outs[j]) for j in range(K)]
            for s in range(2)]

    variants = {
        "single_1M": (1, lambda i: e4.checksum_batch(ds[i % (2 * K)], n=n, stride=L, seg_len=L,
                                                       init=inits[i % (2 * K)], out=outs[0])),
        "single_8M": (K, lambda i: e4.checksum_batch(big[(i % 2) * K * n * L:], n=K * n, stride=L, seg_len=L,
                                                       init=binit[(i % 2) * K * n:], out=bout)),
        "single_1M_segs8": (1, lambda i: s8.checksum_batch(ds[i % (2 * K)], n=n, stride=L, seg_len=L,
                                                             init=inits[i % (2 * K)], out=outs[0])),
        "single_8M_segs8": (K, lambda i: s8.checksum_batch(big[(i % 2) * K * n * L:], n=K * n, stride=L, seg_len=L,
                                                             init=binit[(i % 2) * K * n:], out=bout)),
        "batchv8": (K, lambda i: e4.checksum_batchv(sets[i % 2])),
    }
    # outputs agree: set 0 through every variant
    ref = [t.clone() for t in e4.checksum_batchv(sets[0])]
    for e in (e4,):
        got = e.checksum_batchv(sets[0])
        assert all(torch.equal(a, b) for a, b in zip(got, ref))
    e4.checksum_batch(big, n=K * n, stride=L, seg_len=L, init=binit, out=bout)
    assert torch.equal(bout.view(K, n), torch.stack(ref))
    for name, (per, fn) in variants.items():  # warm
        for i in range(8):
            fn(i)
    torch.cuda.synchronize()
    ts = {k: [] for k in variants}
    for r in range(args.rounds):
        order = list(variants) if r % 2 == 0 else list(reversed(variants))
        for name in order:
            per, fn = variants[name]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for i in range(args.iters):
                fn(i)
            b.record()
            torch.cuda.synchronize()
            ts[name].append(a.elapsed_time(b) / 1e3 / args.iters / per)
    for name in variants:
        t = statistics.median(ts[name])
        print(json.dumps({"variant": name, "us_per_1M_batch": round(t * 1e6, 2),
                          "frac_hbm_peak": round(n * L / t / 1e9 / 8000.0, 4),
                          "all_us": [round(x * 1e6, 2) for x in ts[name]]}), flush=True)


if __name__ == "__main__":
    main()
