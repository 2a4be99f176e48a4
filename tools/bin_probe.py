"""Dev probe: mixed-length offsets batches through the binned and the
single-geometry dispatch (run under rocprofv3 --kernel-trace to split the
time per bin kernel).  The dispatch comes from ICSUM_FORCE in the environment
(e.g. bin=0 / bin=1,bin_blocks=8192).

    python tools/bin_probe.py {mixed|long|bimodal|mss|ack} [iters]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tcpip_network_protocol_stack_amd.engine import Engine, mixed_offsets  # noqa: E402


def main():
    kind = sys.argv[1]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n, seed = 1 << 20, 0x10710004
    off = mixed_offsets(n, seed).astype(np.int64)
    lens = np.diff(off)
    if kind == "long":  # only the segments of the last bin (> 4 KiB), packed
        lens = lens[lens > 4096]
    elif kind in ("mss", "ack"):  # one bin's worth: 1 M x 1460-1463 B or 40-43 B
        rng = np.random.default_rng(seed)
        lens = (1460 if kind == "mss" else 40) + rng.integers(0, 4, n)
    elif kind == "bimodal":
        rng = np.random.default_rng(seed)
        lens = np.where(rng.random(2 * n) < 0.5, 40, 1460) + rng.integers(0, 4, 2 * n)
    off = np.zeros(lens.size + 1, dtype=np.int64)
    off[1:] = np.cumsum(lens)
    eng = Engine(0)
    dev = torch.device("cuda", 0)
    d = eng.fill_bytes(torch.empty(int(off[-1]) + 16, dtype=torch.uint8, device=dev), seed)
    doff = torch.from_numpy(off).to(dev)
    out = torch.empty(lens.size, dtype=torch.int16, device=dev)
    for _ in range(iters):
        eng.checksum_batch(d, offsets=doff, out=out)
    torch.cuda.synchronize()
    print(kind, lens.size, int(off[-1]))


if __name__ == "__main__":
    main()
