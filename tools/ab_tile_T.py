#!/usr/bin/env python3
"""Dev measurement: tile size T of the tile launch (ICSUM_FORCE tile=1,
tile_segs=T) per batch size and mean length — checksum of offsets batches
(0..1000-byte payload datagrams = the transmit mix, a constant 770 B) and the
headers-apart wrap of 0..1000-byte payloads (the stack row's shape).  Two
copies rotate; HIP events around 20 back-to-back calls, median of 5 rounds.
Arguments: sizes (default 196608,262144,524288,1048576), tile sizes
(default 64,96,128,160,192,256)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _force import engine  # noqa: E402
from ab_stack import R, timed, tx_batch  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK = 8.0e12


def main():
    sizes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [196608, 262144, 524288, 1048576]
    Ts = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [64, 96, 128, 160, 192, 256]
    auto = engine()
    engs = {"auto": auto, **{f"T{T}": engine(tile=1, tile_segs=T) for T in Ts}}
    for n in sizes:
        tx = [tx_batch(auto, n, 21 + r) for r in range(R)]
        nb = tx[0][3]
        pb = int(tx[0][5][-1].item()) + 40 * n
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        hd = torch.empty(n * 40, dtype=torch.uint8, device="cuda")
        rng = np.random.default_rng(n)
        lens = np.full(n, 770, dtype=np.uint64)
        off = np.zeros(n + 1, dtype=np.uint64)
        off[1:] = np.cumsum(lens)
        u = [(auto.fill_bytes(torch.empty(int(off[-1]) + 16, dtype=torch.uint8, device="cuda"), 5 + r),
              torch.from_numpy(off.view(np.int64)).cuda()) for r in range(R)]
        del rng
        for name, e in engs.items():
            rows = (("tx_checksum", nb, lambda i, e=e: e.checksum_batch(tx[i % R][0], n=n, offsets=tx[i % R][1], out=out)),
                    ("u770_checksum", int(off[-1]), lambda i, e=e: e.checksum_batch(u[i % R][0], n=n, offsets=u[i % R][1],
                                                                                    out=out)),
                    ("tx_wrap_apart", pb, lambda i, e=e: e.tcp_wrap_headers(tx[i % R][4], tx[i % R][2], hd, n=n,
                                                                            offsets=tx[i % R][5])))
            for row, b, fn in rows:
                t = timed(fn)
                print(json.dumps({"row": f"{row}_{n}", "lib": name, "bytes": b, "us": round(t * 1e6, 2),
                                  "frac": round(b / t / PEAK, 4), "kernel": e.dispatch_info()["kernel"]}), flush=True)
        del tx, u


if __name__ == "__main__":
    main()
