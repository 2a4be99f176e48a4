#!/usr/bin/env python3
"""Dev measurement: the automatic dispatch of offsets batches against the tile
launch (ICSUM_FORCE tile=1), per entry point and length mix, to set the
dispatch rule (icsum_dispatch.cpp, tile_wins).  Mixes: the receive mix (half
40-byte ACKs, half 1500-byte datagrams), 40..1040-byte datagrams (0..1000-byte
payloads), a constant 770 B, MTU (1500 B), pure ACKs (40 B) and the log-uniform
64 B..64 KiB mix of config 4.  Every batch is raw IPv4/TCP datagrams with valid
headers, so the same bytes serve checksum, VERIFY and the wraps.  Two copies
rotate (three for batches under 128 MB); HIP events around back-to-back calls.
Argument: comma-separated batch sizes (default 65536,262144,1048576)."""
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


def timed(fn, iters=20, rounds=5):
    st = torch.cuda.current_stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.1:
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


def lengths(mix, n, rng):
    if mix == "rx":
        return np.where(rng.random(n) < 0.5, 40, 1500)
    if mix == "tx":
        return 40 + rng.integers(0, 1001, n)
    if mix == "u770":
        return np.full(n, 770)
    if mix == "mtu":
        return np.full(n, 1500)
    if mix == "ack":
        return np.full(n, 40)
    # config 4's log-uniform 64 B .. 64 KiB
    return np.floor(np.exp(rng.uniform(np.log(64), np.log(65537), n))).astype(np.int64).clip(64, 65536)


def batch(eng, lens, seed):
    off = np.zeros(lens.size + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    d = eng.fill_bytes(torch.empty(int(off[-1]) + 16, dtype=torch.uint8, device="cuda"), seed)
    # valid headers: ver 4, hlen 5, len, DF, ttl 64, TCP, data offset 5 (device-side: the spec generator
    # writes a fixed stride only, so set the bytes from the host for the starts)
    s = torch.from_numpy(off[:-1].astype(np.int64)).cuda()
    ln = torch.from_numpy(lens.astype(np.int64)).cuda()
    d[s] = 0x45
    d[s + 1] = 0
    d[s + 2] = (ln >> 8).to(torch.uint8)
    d[s + 3] = (ln & 255).to(torch.uint8)
    d[s + 6] = 0x40
    d[s + 7] = 0
    d[s + 8] = 64
    d[s + 9] = 6
    big = s[ln >= 40]
    d[big + 32] = 0x50
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    eng.ipv4_tcp_batch(d, 2, n=lens.size, offsets=doff)  # PATCH: valid checksums
    return d, doff, int(off[-1])


def main():
    sizes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1 << 16, 1 << 18, 1 << 20]
    engs = {"auto": engine(), "tile": engine(tile=1)}
    rng = np.random.default_rng(9)
    for n in sizes:
        m = np.zeros(n, dtype=TCP_MSG_DTYPE)
        for f, hi in (("src", 2**32), ("dst", 2**32), ("seqno", 2**32), ("ackno", 2**32), ("src_port", 2**16),
                      ("dst_port", 2**16), ("window", 2**16)):
            m[f] = rng.integers(0, hi, n, dtype=np.uint64)
        m["flags"], m["ttl"] = 0x10, 128
        dm = torch.from_numpy(m.view(np.uint8).copy()).cuda()
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        ip = torch.empty(n, dtype=torch.int16, device="cuda")
        tcp = torch.empty(n, dtype=torch.int16, device="cuda")
        st = torch.empty(n, dtype=torch.uint8, device="cuda")
        hd = torch.empty(n * 40, dtype=torch.uint8, device="cuda")
        for mix in ("rx", "tx", "u770", "mtu", "ack", "c4"):
            if mix == "c4" and n > (1 << 18):
                continue  # 10 GB at 1 M: config 4 itself is bench_configs' row
            lens = lengths(mix, n, rng)
            nbytes = int(lens.sum())
            R = 2 if nbytes > (128 << 20) else 3
            bs = [batch(engs["auto"], lens, 100 + r) for r in range(R)]
            pl = np.maximum(lens - 40, 0)
            poff = np.zeros(n + 1, dtype=np.uint64)
            poff[1:] = np.cumsum(pl)
            pdoff = torch.from_numpy(poff.view(np.int64)).cuda()
            for name, e in engs.items():
                ops = {
                    "checksum": lambda i, e=e: e.checksum_batch(bs[i % R][0], n=n, offsets=bs[i % R][1], out=out),
                    "verify": lambda i, e=e: e.ipv4_tcp_batch(bs[i % R][0], 1, n=n, offsets=bs[i % R][1], ip_ck=ip,
                                                              tcp_ck=tcp, status=st),
                    "wrap": lambda i, e=e: e.tcp_wrap_batch(bs[i % R][0], dm, n=n, offsets=bs[i % R][1]),
                    # payload arenas: the same buffers read as payload-only batches (poff <= off)
                    "wrap_apart": lambda i, e=e: e.tcp_wrap_headers(bs[i % R][0], dm, hd, n=n, offsets=pdoff),
                }
                for op, fn in ops.items():
                    nb = int(poff[-1]) + 40 * n if op == "wrap_apart" else nbytes
                    t = timed(fn)
                    info = e.dispatch_info()
                    print(json.dumps({"n": n, "mix": mix, "op": op, "eng": name, "bytes": nb, "us": round(t * 1e6, 2),
                                      "frac": round(nb / t / PEAK, 4), "kernel": info["kernel"],
                                      "plan": info["plan"]}), flush=True)
            # the wraps rewrote headers: VERIFY above ran first on every engine
            del bs


if __name__ == "__main__":
    main()
