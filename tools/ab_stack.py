#!/usr/bin/env python3
"""Dev measurement: the stack-tick shapes — 256 Ki received
datagrams (half 40-byte ACKs, half 1500-byte segments, packed offsets) through
VERIFY, and 256 Ki transmitted datagrams (40 bytes of header room + 0..1000
payload bytes, packed) through the in-place wrap — under the automatic
dispatch and forced shapes, beside the plain checksum of the same bytes and
fixed-stride batches of the same volume.  Two copies of each batch rotate, so
no call finds the previous one's bytes in the 256 MiB Infinity Cache.
Times: HIP events around `iters` back-to-back calls, median of 5 rounds."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _force import engine  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tcpip_network_protocol_stack_amd.engine import TCP_MSG_DTYPE  # noqa: E402

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


def emit(name, nbytes, t, **kw):
    print(json.dumps({"row": name, "bytes": nbytes, "us": round(t * 1e6, 2),
                      "frac": round(nbytes / t / PEAK, 4), **kw}), flush=True)


def rx_batch(eng, n, seed):
    rng = np.random.default_rng(seed)
    lens = np.where(rng.random(n) < 0.5, 40, 1500).astype(np.uint64)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    s = off[:-1].astype(np.int64)
    buf[s], buf[s + 1], buf[s + 2], buf[s + 3] = 0x45, 0, (lens >> 8).astype(np.uint8), (lens & 255).astype(np.uint8)
    buf[s + 6], buf[s + 7], buf[s + 8], buf[s + 9], buf[s + 32] = 0x40, 0, 64, 6, 0x50
    d = torch.from_numpy(buf).cuda()
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    eng.ipv4_tcp_batch(d, 2, n=n, offsets=doff)  # PATCH: valid checksums
    return d, doff, int(off[-1])


def tx_batch(eng, n, seed):
    rng = np.random.default_rng(seed)
    pl = rng.integers(0, 1001, n)
    tl = 40 + pl
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(tl)
    poff = np.zeros(n + 1, dtype=np.uint64)
    poff[1:] = np.cumsum(pl)
    d = eng.fill_bytes(torch.empty(int(off[-1]) + 16, dtype=torch.uint8, device="cuda"), seed)
    pd = eng.fill_bytes(torch.empty(int(poff[-1]) + 16, dtype=torch.uint8, device="cuda"), seed + 7)
    m = np.zeros(n, dtype=TCP_MSG_DTYPE)
    for f, hi in (("src", 2**32), ("dst", 2**32), ("seqno", 2**32), ("ackno", 2**32), ("src_port", 2**16),
                  ("dst_port", 2**16), ("window", 2**16)):
        m[f] = rng.integers(0, hi, n, dtype=np.uint64)
    m["flags"], m["ttl"] = 0x10, 128
    dm = torch.from_numpy(m.view(np.uint8).copy()).cuda()
    return d, torch.from_numpy(off.view(np.int64)).cuda(), dm, int(off[-1]), pd, torch.from_numpy(poff.view(np.int64)).cuda()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
    auto = engine()
    shapes = {"auto": auto, "twoclass32": engine(twoclass=32), "l16u4": engine(lps=16, unroll=4, mode=3),
              "l16u8": engine(lps=16, unroll=8, mode=3), "l8u8": engine(lps=8, unroll=8, mode=3),
              "l4u2m2": engine(lps=4, unroll=2, mode=2), "tile": engine(tile=1),
              "tile64": engine(tile=1, tile_segs=64), "tile128": engine(tile=1, tile_segs=128),
              "tile256": engine(tile=1, tile_segs=256), "auto_x10": engine(twoclass_remap=10),
              "auto_x6": engine(twoclass_remap=6)}
    tiles = ("tile", "tile64", "tile128", "tile256")
    rx = [rx_batch(auto, n, 11 + r) for r in range(R)]
    nb = rx[0][2]
    ip = torch.empty(n, dtype=torch.int16, device="cuda")
    tcp = torch.empty(n, dtype=torch.int16, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    for name, e in shapes.items():
        t = timed(lambda i, e=e: e.ipv4_tcp_batch(rx[i % R][0], 1, n=n, offsets=rx[i % R][1], ip_ck=ip, tcp_ck=tcp,
                                                  status=st))
        assert (st.cpu().numpy() == 0x0F).all(), name
        emit(f"verify_{name}", nb, t, kernel=e.dispatch_info()["kernel"])
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    for name in ("auto", "twoclass32", "l16u4", "auto_x10", "auto_x6") + tiles:
        e = shapes[name]
        t = timed(lambda i, e=e: e.checksum_batch(rx[i % R][0], n=n, offsets=rx[i % R][1], out=out))
        emit(f"plain_rx_{name}", nb, t, kernel=e.dispatch_info()["kernel"])
    del rx
    # the same volume at a fixed stride: 770 B (the mean) and 1500 B (the MTU half)
    for L, m in ((770, n), (1500, n // 2)):
        ds = [auto.fill_bytes(torch.empty(m * L, dtype=torch.uint8, device="cuda"), 5, pos0=r * m * L)
              for r in range(R)]
        t = timed(lambda i: auto.checksum_batch(ds[i % R], n=m, stride=L, seg_len=L, out=out))
        emit(f"plain_fixed_{m}x{L}", m * L, t, kernel=auto.dispatch_info()["kernel"])
        del ds
    tx = [tx_batch(auto, n, 21 + r) for r in range(R)]
    nb = tx[0][3]
    for name in ("auto", "l16u4", "l16u8", "l8u8", "l4u2m2") + tiles:
        e = shapes[name]
        t = timed(lambda i, e=e: e.tcp_wrap_batch(tx[i % R][0], tx[i % R][2], n=n, offsets=tx[i % R][1]))
        emit(f"wrap_{name}", nb, t, kernel=e.dispatch_info()["kernel"], lps=e.dispatch_info()["lps"])
    for name in ("auto", "l16u4") + tiles:
        e = shapes[name]
        t = timed(lambda i, e=e: e.checksum_batch(tx[i % R][0], n=n, offsets=tx[i % R][1], out=out))
        emit(f"plain_tx_{name}", nb, t, kernel=e.dispatch_info()["kernel"])
    # headers apart (the iovec form): payloads alone, 40 header bytes per datagram into one array
    hd = torch.empty(n * 40, dtype=torch.uint8, device="cuda")
    apart = dict(shapes)
    apart.update({"tile_2p": engine(tile=1, wrap_passes=2), "auto_2p": engine(wrap_passes=2),
                  "auto_1p": engine(wrap_passes=1)})
    for name in ("auto", "auto_1p", "auto_2p", "tile_2p", "l16u4"):
        e = apart[name]
        t = timed(lambda i, e=e: e.tcp_wrap_headers(tx[i % R][4], tx[i % R][2], hd, n=n, offsets=tx[i % R][5]))
        emit(f"wrap_apart_{name}", nb, t, kernel=e.dispatch_info()["kernel"], lps=e.dispatch_info()["lps"])


if __name__ == "__main__":
    main()
