#!/usr/bin/env python3
"""Dev measurement: the tile launch (k_tile) across tile sizes and grid caps,
on three offsets batches of about the same volume — the receive mix (half
40-byte ACKs, half 1500-byte segments), uniform 0..1000-byte payloads, and a
constant 770-byte length given as offsets — beside the fixed-stride kernel
over the same 770-byte batch (the streaming reference).  Two copies rotate;
HIP events around 20 back-to-back calls, median of 5 rounds.
Argument: batch size in segments (default 256 Ki)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _force import engine  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK = 8.0e12
R = 2


def timed(fn, iters=20, rounds=5):
    st = torch.cuda.current_stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.15:
        for i in range(8):
            fn(i)
        torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for i in range(iters):
            fn(i)
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 1e3 / iters)
    return statistics.median(ts)


def batch(eng, lens, seed):
    off = np.zeros(lens.size + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    d = eng.fill_bytes(torch.empty(int(off[-1]) + 16, dtype=torch.uint8, device="cuda"), seed)
    return d, torch.from_numpy(off.view(np.int64)).cuda(), int(off[-1])


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
    auto = engine()
    rng = np.random.default_rng(3)
    mixes = {"rx": np.where(rng.random(n) < 0.5, 40, 1500), "tx": rng.integers(0, 1001, n),
             "u770": np.full(n, 770)}
    variants = {"auto": {}}
    for T in (64, 128, 256):
        for blocks in (0, 1024):  # one block per tile; persistent (the 1024 resident blocks)
            variants[f"T{T}_b{blocks}"] = {"tile": 1, "tile_segs": T, "tile_blocks": blocks}
    engs = {k: engine(**v) for k, v in variants.items()}
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    for mix, lens in mixes.items():
        bs = [batch(auto, lens, 11 + r) for r in range(R)]
        nb = bs[0][2]
        for name, e in engs.items():
            t = timed(lambda i, e=e: e.checksum_batch(bs[i % R][0], n=n, offsets=bs[i % R][1], out=out))
            print(json.dumps({"row": f"{mix}_{name}", "bytes": nb, "us": round(t * 1e6, 2),
                              "frac": round(nb / t / PEAK, 4), "kernel": e.dispatch_info()["kernel"]}), flush=True)
        del bs
    ds = [auto.fill_bytes(torch.empty(n * 770, dtype=torch.uint8, device="cuda"), 5, pos0=r * n * 770)
          for r in range(R)]
    t = timed(lambda i: auto.checksum_batch(ds[i % R], n=n, stride=770, seg_len=770, out=out))
    print(json.dumps({"row": "fixed_770", "bytes": n * 770, "us": round(t * 1e6, 2),
                      "frac": round(n * 770 / t / PEAK, 4)}), flush=True)


if __name__ == "__main__":
    main()
