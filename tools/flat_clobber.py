#!/usr/bin/env python3
"""Dev tool: ab_lastbin's call sequence on config 4 (default dispatch into
out0, then the flat dispatch into out1, both preallocated) with host copies
in between: does the flat call disturb out0, and where do they differ."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tcpip_network_protocol_stack_amd.engine import Engine, mixed_offsets  # noqa: E402


def engine(env):
    os.environ.update(env)
    try:
        return Engine(0)
    finally:
        for k in env:
            del os.environ[k]


def main():
    dev = torch.device("cuda", 0)
    e0, e1 = engine({"ICSUM_FLAT": "0"}), engine({"ICSUM_FLAT": "1"})
    off = mixed_offsets(1 << 20, 0x10710004).astype(np.int64)
    d = e0.fill_bytes(torch.empty(int(off[-1]) + 16, dtype=torch.uint8, device=dev), 0x10710004)
    toff = torch.from_numpy(off).to(dev)
    n = off.size - 1
    out0 = torch.empty(n, dtype=torch.int16, device=dev)
    out1 = torch.empty(n, dtype=torch.int16, device=dev)
    print(json.dumps({"out0": out0.data_ptr(), "out1": out1.data_ptr(), "d": d.data_ptr()}), flush=True)
    e0.checksum_batch(d, offsets=toff, out=out0)
    torch.cuda.synchronize()
    h0 = out0.cpu().numpy().copy()
    e1.checksum_batch(d, offsets=toff, out=out1)
    torch.cuda.synchronize()
    h0b, h1 = out0.cpu().numpy(), out1.cpu().numpy()
    for name, a, b in (("out0_before_vs_after", h0, h0b), ("auto_vs_flat", h0, h1), ("auto_after_vs_flat", h0b, h1)):
        bad = np.flatnonzero(a != b)
        rows = [{"j": int(j), "s": int(off[j]), "len": int(off[j + 1] - off[j]), "a": int(a[j]), "b": int(b[j])}
                for j in bad[:8]]
        print(json.dumps({"cmp": name, "mismatches": int(bad.size), "first": rows}), flush=True)
    e2 = engine({"ICSUM_FLAT": "1"})
    out2 = e2.checksum_batch(d, offsets=toff).cpu().numpy()
    print(json.dumps({"cmp": "fresh_flat_vs_auto", "mismatches": int((out2 != h0).sum())}), flush=True)


if __name__ == "__main__":
    main()
