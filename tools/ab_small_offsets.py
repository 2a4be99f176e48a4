#!/usr/bin/env python3
"""Dev A/B: device-resident OFFSETS batches below the binning threshold
(bin_min, 64 Ki segments) run as one launch, its geometry from the plan
cache.  Compares, interleaved in one process: the default, a lower bin_min
(ICSUM_FORCE bin_min=1024: binning + the plan cache, so repeat calls on the
same offsets run the cached plan's single launch), binning on every call
(bin=1: no plan cache), and the best fixed geometry for
the length (forced), for 4-32 Ki segments of 64 / 576 / 1500 bytes."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from _force import engine  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    engs = {"default": engine(), "binmin1k": engine(bin_min=1024), "binned_nocache": engine(bin=1)}
    for n in (8192, 16384, 32768, 65535):
        for L in (64, 576, 1500):
            R = max(2, (400 << 20) // (n * L) + 1)
            off = np.arange(n + 1, dtype=np.int64) * L
            doff = torch.from_numpy(off).to(dev)
            ds = [engs["default"].fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), 7, pos0=r * n * L)
                  for r in range(R)]
            out = torch.empty(n, dtype=torch.int16, device=dev)
            res = {}
            for k, e in engs.items():
                fn = lambda i, e=e: e.checksum_batch(ds[i % R], offsets=doff, out=out)  # noqa: E731
                ts = []
                for rnd in range(5):
                    t0 = time.perf_counter()
                    while time.perf_counter() - t0 < 0.02:
                        for i in range(4):
                            fn(i)
                        torch.cuda.synchronize()
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for i in range(40):
                        fn(i)
                    b.record()
                    torch.cuda.synchronize()
                    ts.append(a.elapsed_time(b) * 1e3 / 40)
                res[k] = round(float(np.median(ts)), 2)
            fixed = engs["default"].checksum_batch
            ts = []
            for rnd in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for i in range(40):
                    fixed(ds[i % R], n=n, stride=L, seg_len=L, out=out)
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3 / 40)
            res["fixed_stride_reference"] = round(float(np.median(ts)), 2)
            print(json.dumps({"n": n, "L": L, **res}), flush=True)
            del ds


if __name__ == "__main__":
    main()
