#!/usr/bin/env python3
"""Dev tool: config 4 at full size (pseudo-header inits) through the default
dispatch and the flat dispatch, many calls each, every output's SHA-256
against the reference digest (tests/golden/configs.json "4")."""
import hashlib
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))["4"]
    n, seed = g["n"], g["seed"]
    dev = torch.device("cuda", 0)
    engs = {"auto": engine({"ICSUM_FLAT": "0"}), "flat16384": engine({"ICSUM_FLAT": "1"}),
            "flat6144": engine({"ICSUM_FLAT": "1", "ICSUM_FLAT_WAVES": "6144"})}
    base = engs["auto"]
    off = mixed_offsets(n, seed)
    data = base.fill_bytes(torch.empty(int(off[-1]), dtype=torch.uint8, device=dev), seed)
    doff = torch.from_numpy(off.view(np.int64)).to(dev)
    init = base.pseudo_inits(n, seed, offsets=doff)
    torch.cuda.synchronize()
    for name, eng in engs.items():
        ok, bad = 0, []
        for r in range(reps):
            out = eng.checksum_batch(data, offsets=doff, init=init).cpu().numpy()
            h = hashlib.sha256(out.tobytes()).hexdigest()
            if h == g["out_sha256"]:
                ok += 1
            else:
                bad.append(r)
        print(json.dumps({"engine": name, "calls": reps, "match_reference": ok, "bad_calls": bad}), flush=True)


if __name__ == "__main__":
    main()
