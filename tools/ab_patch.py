#!/usr/bin/env python3
"""Dev tool: interleaved in-process A/B of the ICS_MODE_PATCH field-store
policy on BASELINE config 2 (64 Ki x 1500 B IPv4 datagrams, 6 rotated copies
so every launch reads HBM): write-back (ICSUM_PATCH_WT=0) vs write-through
(ICSUM_PATCH_WT=1, sc1), with COMPUTE (no stores into the datagrams) as the
floor.  Both patch variants must leave identical bytes that VERIFY accepts.

    python tools/ab_patch.py [--rounds 9] [--iters 60]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from tcpip_network_protocol_stack_amd.engine import Engine  # noqa: E402


def engine(wt):
    os.environ["ICSUM_PATCH_WT"] = str(wt)
    try:
        return Engine(0)
    finally:
        del os.environ["ICSUM_PATCH_WT"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=60)
    args = ap.parse_args()
    n, L, seed, R = 1 << 16, 1500, 0x10710002, 6
    dev = torch.device("cuda", 0)
    wb, wt = engine(0), engine(1)
    bufs = []
    for r in range(R):
        d = wb.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L)
        wb.ipv4_tcp_headers(d, n, L, L, seed, index0=r * n)
        bufs.append(d)
    ip = torch.empty(n, dtype=torch.int16, device=dev)
    tcp = torch.empty(n, dtype=torch.int16, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)

    # same bytes out of both policies, and VERIFY accepts them
    a, b = bufs[0].clone(), bufs[0].clone()
    wb.ipv4_tcp_batch(a, 2, n=n, stride=L, dgram_len=L)
    wt.ipv4_tcp_batch(b, 2, n=n, stride=L, dgram_len=L)
    _, _, ok = wb.ipv4_tcp_batch(b, 1, n=n, stride=L, dgram_len=L)
    torch.cuda.synchronize()
    assert torch.equal(a, b), "write-back and write-through patches differ"
    assert bool((ok == 0x0F).all()), "patched datagrams do not verify"
    del a, b

    variants = [("compute", wb, 0), ("patch_wb", wb, 2), ("patch_wt", wt, 2)]

    def run(eng, mode, k):
        eng.ipv4_tcp_batch(bufs[k % R], mode, n=n, stride=L, dgram_len=L, ip_ck=ip, tcp_ck=tcp, status=st)

    t0 = time.perf_counter()  # settle the clocks (bench.py --settle-ms)
    while time.perf_counter() - t0 < 0.3:
        for k in range(16):
            run(wb, 0, k)
        torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    times = {v[0]: [] for v in variants}
    for r in range(args.rounds):
        for name, eng, mode in variants if r % 2 == 0 else variants[::-1]:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for k in range(args.iters):
                run(eng, mode, k)
            e1.record(s)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) * 1e3 / args.iters)
    for name, ts in times.items():
        med = statistics.median(ts)
        print(json.dumps({"config": "ipv4_64Kix1500", "variant": name, "med_us": round(med, 2),
                          "min_us": round(min(ts), 2), "GB_s": round(n * L / med / 1e3, 1),
                          "frac_hbm_peak": round(n * L / med / 1e3 / 8000.0, 4)}), flush=True)
    wb.close()
    wt.close()


if __name__ == "__main__":
    main()
