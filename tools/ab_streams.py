#!/usr/bin/env python3
"""Dev A/B: a stream of short batches (configs 2 and 3) issued on 1, 2 or 4
HIP streams in turn.  One stream pays every launch's ramp and drain in
series; with several, batch i+1's waves start while batch i's last waves
drain.  Per-batch time = (last batch done - first issued) / batches, each
stream with its own output arrays; rotated input copies as in
tools/bench_configs.py."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from tcpip_network_protocol_stack_amd.engine import Engine  # noqa: E402

PEAK = 8.0e12


def run(fn, k, streams, iters=60, rounds=5):
    """fn(i, stream, slot) issues batch i; returns median seconds per batch."""
    main = torch.cuda.current_stream()
    ts = []
    for r in range(rounds + 1):
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        start.record(main)
        for s in streams[:k]:
            s.wait_stream(main)
        for i in range(iters):
            j = i % k
            fn(i, streams[j], j)
        for s in streams[:k]:
            main.wait_stream(s)
        end.record(main)
        torch.cuda.synchronize()
        if r:  # the first round settles clocks
            ts.append(start.elapsed_time(end) / 1e3 / iters)
    return statistics.median(ts)


def main():
    eng = Engine(0)
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    warm = eng.fill_bytes(torch.empty(1 << 30, dtype=torch.uint8, device=dev), 1)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2:
        eng.checksum_batch(warm, n=1 << 20, stride=1024, seg_len=1024)
        torch.cuda.synchronize()
    del warm

    n, L, seed, R = 1 << 16, 1500, 0x10710002, 6
    bufs = []
    for r in range(R):
        d = eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L)
        eng.ipv4_tcp_headers(d, n, L, L, seed, index0=r * n)
        eng.ipv4_tcp_batch(d, 2, n=n, stride=L, dgram_len=L)
        bufs.append(d)
    outs = [(torch.empty(n, dtype=torch.int16, device=dev), torch.empty(n, dtype=torch.int16, device=dev),
             torch.empty(n, dtype=torch.uint8, device=dev)) for _ in range(4)]
    for mode, nm in ((0, "compute"), (1, "verify")):
        for k in (1, 2, 4):
            t = run(lambda i, s, j: eng.ipv4_tcp_batch(bufs[i % R], mode, n=n, stride=L, dgram_len=L,
                                                      ip_ck=outs[j][0], tcp_ck=outs[j][1], status=outs[j][2],
                                                      stream=s), k, streams)
            print(json.dumps({"config": f"ipv4_64Kix1500_{nm}", "streams": k, "us": round(t * 1e6, 2),
                              "frac_hbm_peak": round(n * L / t / PEAK, 4)}), flush=True)
    for k in (1, 2, 4):
        t = run(lambda i, s, j: eng.checksum_batch(bufs[i % R], n=n, stride=L, seg_len=L, out=outs[j][0], stream=s),
                k, streams)
        print(json.dumps({"config": "plain_64Kix1500", "streams": k, "us": round(t * 1e6, 2),
                          "frac_hbm_peak": round(n * L / t / PEAK, 4)}), flush=True)
    del bufs

    n, L, seed = 1 << 20, 64, 0x10710003
    ds = [eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L) for r in range(R)]
    inits = [eng.pseudo_inits(n, seed, seg_len=L, index0=r * n) for r in range(R)]
    o16 = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(4)]
    for k in (1, 2, 4):
        t = run(lambda i, s, j: eng.checksum_batch(ds[i % R], n=n, stride=L, seg_len=L, init=inits[i % R], out=o16[j],
                                                  stream=s), k, streams)
        print(json.dumps({"config": "tcp_1Mx64", "streams": k, "us": round(t * 1e6, 2),
                          "frac_hbm_peak": round(n * L / t / PEAK, 4)}), flush=True)


if __name__ == "__main__":
    main()
