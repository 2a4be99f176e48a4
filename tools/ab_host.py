#!/usr/bin/env python3
"""Dev tool: interleaved in-process A/B of the host-memory pipeline's staging
(ICSUM_HOST_SLOTS slots of ICSUM_HOST_SLOT_MB each) on the PCIe-inclusive
row of tools/bench_configs.py (256 Ki x 1500 B from pinned and from pageable
host memory, u16 results back), next to a bare H2D copy of the same bytes.

    python tools/ab_host.py [--variants 2x64,3x32,4x32,4x16] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tcpip_network_protocol_stack_amd.engine import Engine  # noqa: E402


def engine(slots, mb):
    env = {"ICSUM_HOST_SLOTS": str(slots), "ICSUM_HOST_SLOT_MB": str(mb)}
    os.environ.update(env)
    try:
        return Engine(0)
    finally:
        for k in env:
            del os.environ[k]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="2x64,3x32,4x32,4x16")
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    from oracle import oracle as orc  # workload bytes only (spec generator)

    n, L, seed = 1 << 18, 1500, 0x10710000
    variants = [(int(v.split("x")[0]), int(v.split("x")[1])) for v in args.variants.split(",")]
    engs = {v: engine(*v) for v in variants}
    bufs = {}
    for pinned in (True, False):
        h = torch.empty(n * L, dtype=torch.uint8, pin_memory=pinned)
        h.numpy()[:] = orc.fill_bytes(seed, 0, n * L)
        bufs[pinned] = h
    init = np.array([orc.pseudo_init(seed, i, L) for i in range(n)], dtype=np.uint32)
    ref = None
    for v, e in engs.items():  # warm (allocates the staging) and check
        out = e.checksum_batch_host(bufs[True].numpy(), n, stride=L, seg_len=L, init=init)
        ref = out if ref is None else ref
        assert (out == ref).all(), v
    d = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    times = {(v, p): [] for v in variants for p in (True, False)}
    copy_ts = []
    for r in range(args.rounds):
        for v in variants if r % 2 == 0 else variants[::-1]:
            for p in (True, False):
                t0 = time.perf_counter()
                engs[v].checksum_batch_host(bufs[p].numpy(), n, stride=L, seg_len=L, init=init)
                times[(v, p)].append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        d.copy_(bufs[True], non_blocking=True)
        torch.cuda.synchronize()
        copy_ts.append(time.perf_counter() - t0)
    for (v, p), ts in times.items():
        med = statistics.median(ts)
        print(json.dumps({"slots": v[0], "slot_MB": v[1], "pinned": p, "med_ms": round(med * 1e3, 3),
                          "GB_s": round(n * L / med / 1e9, 2)}), flush=True)
    med = statistics.median(copy_ts)
    print(json.dumps({"bare_h2d_copy": True, "med_ms": round(med * 1e3, 3), "GB_s": round(n * L / med / 1e9, 2)}))


if __name__ == "__main__":
    main()
