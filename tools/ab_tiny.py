#!/usr/bin/env python3
"""Dev tool: the tiny-segment kernel (one lane per segment, ICSUM_FORCE mode=4)
against the AUTO dispatch and the small-segment body on ACK-sized batches
(offsets and fixed stride); outputs compared, median µs per call."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from _force import engine, geometry  # noqa: E402

VARIANTS = {"auto": {}, "tiny": geometry(1, 4, 4), "small4x2s2": geometry(4, 2, 2, segs=2)}


def main():
    dev = torch.device("cuda", 0)
    engs = {k: engine(**v) for k, v in VARIANTS.items()}
    base = engs["auto"]
    rng = np.random.default_rng(0xAC4)
    n = 1 << 20
    cases = []
    for lo, hi in ((40, 44), (20, 64), (64, 145)):
        lens = rng.integers(lo, hi, n)
        off = np.zeros(n + 1, dtype=np.int64)
        off[1:] = np.cumsum(lens)
        cases.append((f"offsets_{lo}_{hi - 1}B", dict(offsets=torch.from_numpy(off).to(dev)), int(off[-1])))
    for L in (40, 52, 64):
        cases.append((f"stride_{L}B", dict(n=n, stride=L, seg_len=L), n * L))
    for name, kw, nbytes in cases:
        d = base.fill_bytes(torch.empty(nbytes + 64, dtype=torch.uint8, device=dev), 0x71)
        outs = {k: e.checksum_batch(d, **kw) for k, e in engs.items()}
        torch.cuda.synchronize()
        for k in engs:
            assert torch.equal(outs[k], outs["auto"]), (name, k)
        times = {k: [] for k in engs}
        st = torch.cuda.current_stream()
        for r in range(5):
            for k, e in engs.items():
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(20):
                    e.checksum_batch(d, out=outs[k], **kw)
                b.record(st)
                torch.cuda.synchronize()
                times[k].append(a.elapsed_time(b) * 1e3 / 20)
        for k, ts in times.items():
            med = statistics.median(ts)
            print(json.dumps({"workload": name, "segments": n, "bytes": nbytes, "variant": k, "med_us": round(med, 2),
                              "GB_s": round(nbytes / med / 1e3, 1)}), flush=True)
        del d


if __name__ == "__main__":
    main()
