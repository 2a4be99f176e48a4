#!/usr/bin/env python3
"""Dev measurement (round 5): the tile launch (k_span, one wave per 63
segments) against the per-segment launches (and, in git c581ecc, against
round 4's k_tile: profiles/r5k_ab_span_ops.jsonl), on the VERDICT r4 shapes — the transmit mix
(payloads of 0..1000 bytes: 40..1040-byte datagrams, or the payloads alone
for the headers-apart wrap) at 256 Ki and 1 M segments, and constant
770-byte segments given as offsets — for the checksum, ics_tcp_wrap_headers
(wrap_apart), the in-place wrap and the fused IPv4 kernel's VERIFY / PATCH
(random bytes: header lengths of 20..60).  Each row: back to back (events
around 20 calls, median of 5 rounds, two batches rotated) and alone (events
around one call after a synchronize, median of 40).  Variants through
ICSUM_FORCE.  Usage: python tools/ab_stream.py [rows] [variants] [ops];
AB_LIGHT=1: a few calls per row (counter passes)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _force import engine  # noqa: E402
from tcpip_network_protocol_stack_amd.engine import mixed_offsets  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK = 8.0e12
R = 2


LIGHT = bool(os.environ.get("AB_LIGHT"))  # counter passes: a few calls per row


def b2b(fn, iters=20, rounds=5):
    if LIGHT:
        iters, rounds = 3, 1
    st = torch.cuda.current_stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < (0.0 if LIGHT else 0.15):
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


def alone(fn, calls=40):
    if LIGHT:
        calls = 2
    st = torch.cuda.current_stream()
    ts = []
    for i in range(calls + 5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record(st)
        fn(i)
        b.record(st)
        torch.cuda.synchronize()
        if i >= 5:
            ts.append(a.elapsed_time(b) / 1e3)
    return statistics.median(ts)


def batch(eng, lens, seed):
    off = np.zeros(lens.size + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    d = eng.fill_bytes(torch.empty(int(off[-1]) + 16, dtype=torch.uint8, device="cuda"), seed)
    return d, torch.from_numpy(off.view(np.int64)).cuda(), int(off[-1])


VARIANTS = {
    "auto": {},                  # the default dispatch
    "span": {"tile": 1},         # the tile launch, k_span (span size: the plan's, or 63)
    "per_segment": {"tile": 0},  # the per-segment / two-class launches
    **{f"S{k}": {"tile": 1, "span_segs": k} for k in range(1, 64)},
    # one per-segment launch of a forced lane-group geometry (g<lanes>x<loads per lane>)
    **{f"g{l}x{u}": {"tile": 0, "lps": l, "unroll": u, "mode": 3} for l, u in ((8, 8), (16, 4), (16, 8), (32, 8))},
    # the span launch as a persistent grid of G blocks (grid-stride over the spans)
    **{f"G{g}": {"span_blocks": g} for g in (768, 1024, 1280, 1536, 2048, 4096)},
}


def main():
    rows = (sys.argv[1] if len(sys.argv) > 1 else "tx256k,tx1m,u770_256k,u770_1m").split(",")
    names = (sys.argv[2] if len(sys.argv) > 2 else ",".join(VARIANTS)).split(",")
    ops = (sys.argv[3] if len(sys.argv) > 3 else "checksum,wrap_apart").split(",")
    engs = {k: engine(**VARIANTS[k]) for k in names}
    auto = engine()
    rng = np.random.default_rng(3)
    shapes = {"tx256k": (1 << 18, "tx"), "tx1m": (1 << 20, "tx"), "u770_256k": (1 << 18, "u770"),
              "u770_1m": (1 << 20, "u770"), "c4_128k": (1 << 17, "c4"), "tx64k": (1 << 16, "tx"),
              "mtu256k": (1 << 18, "mtu"), "mtu1m": (1 << 20, "mtu"), "rx256k": (1 << 18, "rx50"),
              "rx1m25": (1 << 20, "rx25"), "rx1m50": (1 << 20, "rx50"), "rx1m75": (1 << 20, "rx75")}
    for row in rows:
        n, kind = shapes[row]
        if kind.startswith("rx"):  # received traffic: ACKs (40 B) among MTU datagrams, the share in the name
            pays = np.where(rng.random(n) < int(kind[2:]) / 100, 0, 1460)
        elif kind == "c4":  # BASELINE config 4's length mix (64 B - 64 KiB), 128 Ki segments
            pays = np.diff(mixed_offsets(n, 4).astype(np.int64)) - 40
        else:
            pays = rng.integers(0, 1001, n) if kind == "tx" else np.full(n, 1460 if kind == "mtu" else 730)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        hd = torch.empty(n * 40, dtype=torch.uint8, device="cuda")
        msgs = torch.from_numpy(rng.integers(0, 256, n * 28, dtype=np.uint8)).cuda()
        for op in ops:
            lens = pays if op == "wrap_apart" else pays + 40
            bs = [batch(auto, lens, 11 + r) for r in range(R)]
            for d, o, _ in bs:  # IPv4, IHL 5 at every datagram start (the rest random)
                d[o[:-1][torch.from_numpy(lens).cuda() >= 20]] = 0x45
            nb = bs[0][2]
            for name, e in engs.items():
                if op == "checksum":
                    fn = lambda i, e=e: e.checksum_batch(bs[i % R][0], n=n, offsets=bs[i % R][1], out=out)
                elif op == "wrap_apart":
                    fn = lambda i, e=e: e.tcp_wrap_headers(bs[i % R][0], msgs, hd, n=n, offsets=bs[i % R][1])
                elif op == "wrap":
                    fn = lambda i, e=e: e.tcp_wrap_batch(bs[i % R][0], msgs, n=n, offsets=bs[i % R][1])
                else:
                    mode = {"verify": 1, "patch": 2}[op]
                    fn = lambda i, e=e, mode=mode: e.ipv4_tcp_batch(bs[i % R][0], mode, n=n, offsets=bs[i % R][1])
                tb = b2b(fn)
                ta = alone(fn)
                info = e.dispatch_info()
                print(json.dumps({"row": f"{row}_{op}", "variant": name, "bytes": nb, "us_b2b": round(tb * 1e6, 2),
                                  "frac_b2b": round(nb / tb / PEAK, 4), "us_alone": round(ta * 1e6, 2),
                                  "frac_alone": round(nb / ta / PEAK, 4), "kernel": info["kernel"],
                                  "T": info["lps"], "op": info["unroll"]}), flush=True)
            del bs
            torch.cuda.empty_cache()
        # the fixed-stride kernel over the same number of bytes (constant-length
        # rows: the streaming reference a tile launch is measured against)
        if kind in ("u770", "mtu"):
            L = int(pays[0]) + 40
            ds = [auto.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device="cuda"), 5, pos0=r * n * L)
                  for r in range(R)]
            fn = lambda i: auto.checksum_batch(ds[i % R], n=n, stride=L, seg_len=L, out=out)
            tb, ta = b2b(fn), alone(fn)
            print(json.dumps({"row": f"{row}_fixed_stride", "variant": "k_checksum", "bytes": n * L,
                              "us_b2b": round(tb * 1e6, 2), "frac_b2b": round(n * L / tb / PEAK, 4),
                              "us_alone": round(ta * 1e6, 2), "frac_alone": round(n * L / ta / PEAK, 4),
                              "kernel": auto.dispatch_info()["kernel"], "T": 0, "op": 0}), flush=True)
            del ds


if __name__ == "__main__":
    main()
