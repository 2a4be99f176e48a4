"""Dev probe: which segments of a bimodal batch differ from the oracle under
the current ICSUM_BIN* settings (prints mismatch counts per length class)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as orc  # noqa: E402
from tcpip_network_protocol_stack_amd.engine import Engine  # noqa: E402

rng = np.random.default_rng(0xACC)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 150_000
lens = np.where(rng.random(n) < 0.5, 40, 1460) + rng.integers(0, 4, n)
off = np.zeros(n + 1, dtype=np.uint64)
off[1:] = np.cumsum(lens)
off += 1
buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
want = orc.checksum_batch(buf, n, offsets=off)
eng = Engine(0)
dev = torch.device("cuda", 0)
db = torch.from_numpy(buf).to(dev)
do = torch.from_numpy(off.view(np.int64)).to(dev)
for rep in range(3):
    out = eng.checksum_batch(db, offsets=do).cpu().numpy().view(np.uint16)
    bad = out != want
    print(os.environ.get("ICSUM_BIN_PLAN"), os.environ.get("ICSUM_BIN_BLOCKS"), "rep", rep, "bad", int(bad.sum()),
          "short", int((bad & (lens < 100)).sum()), "long", int((bad & (lens > 100)).sum()),
          "first", np.nonzero(bad)[0][:8].tolist(), "zeros_out", int((out[bad] == 0).sum()))
