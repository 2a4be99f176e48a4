#!/usr/bin/env python3
"""Dev tool: where the host-memory wrap (ics_tcp_wrap_batch_host, 256 Ki x
1040-byte datagrams in page-locked memory) spends the time it takes above
the checksum pipeline over the same bytes.  Interleaved, medians of --rounds:

  csum      ics_checksum_batch_host over the same datagrams (u16 back)
  wrap      ics_tcp_wrap_batch_host (40 header bytes written into each datagram)
  headers   ics_tcp_wrap_headers_host over 1000-byte payloads (headers to one array)
  copy      one hipMemcpy of the datagram bytes to the device
  wrap_const7 / wrap_slice / wrap_x5 / wrap_const7_slice_x5: the wrap in
            bench_configs.py's form (constant bytes, records sliced from a
            larger array, five calls back to back; per-call time)

    python tools/ab_wrap_host.py [--rounds 7] [--slots 3] [--slot-mb 32]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tcpip_network_protocol_stack_amd.engine import TCP_MSG_DTYPE, Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--slots", default=None)
    ap.add_argument("--slot-mb", default=None)
    ap.add_argument("--extra-engines", type=int, default=0)
    ap.add_argument("--extra-streams", type=int, default=0)
    ap.add_argument("--cases", default=None, help="comma-separated subset")
    args = ap.parse_args()
    if args.slots:
        os.environ["ICSUM_HOST_SLOTS"] = args.slots
    if args.slot_mb:
        os.environ["ICSUM_HOST_SLOT_MB"] = args.slot_mb
    n, L, P = 1 << 18, 1040, 1000
    # other streams in the process before this engine's: torch streams, and
    # engines whose host staging (their own slot streams) is already set up
    keep = [torch.cuda.Stream() for _ in range(args.extra_streams)]
    for _ in range(args.extra_engines):
        e = Engine(0)
        e.checksum_batch_host(np.zeros(4096, dtype=np.uint8), 1, stride=4096, seg_len=4096)
        e.tcp_wrap_batch_host(np.zeros(1 << 22, dtype=np.uint8), np.zeros(4, dtype=TCP_MSG_DTYPE), 4,
                              stride=1 << 20, dgram_len=1 << 20)
        keep.append(e)
    eng = Engine(0)
    rng = np.random.default_rng(0x10710008)
    m = np.zeros(n, dtype=TCP_MSG_DTYPE)
    for f, hi in (("src", 2**32), ("dst", 2**32), ("seqno", 2**32), ("ackno", 2**32), ("src_port", 2**16),
                  ("dst_port", 2**16), ("window", 2**16)):
        m[f] = rng.integers(0, hi, n, dtype=np.uint64)
    m["flags"], m["ttl"] = 0x10, 64
    dg = torch.empty(n * L, dtype=torch.uint8, pin_memory=True).numpy()
    dg[:] = rng.integers(0, 256, n * L, dtype=np.uint8)
    pl = torch.empty(n * P, dtype=torch.uint8, pin_memory=True).numpy()
    pl[:] = dg.reshape(n, L)[:, 40:].reshape(-1)
    d = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    dgt = torch.from_numpy(dg)
    # bench_configs' form of the row: a buffer of constant bytes, the records a
    # slice of a 1 M-record array, five calls back to back
    big = np.zeros(4 * n, dtype=TCP_MSG_DTYPE)
    big[:n] = m
    dg7 = torch.empty(n * L, dtype=torch.uint8, pin_memory=True).numpy()
    dg7[:] = 7

    def five(buf, msgs):
        for _ in range(5):
            eng.tcp_wrap_batch_host(buf, msgs, n, stride=L, dgram_len=L)

    cases = {
        "csum": lambda: eng.checksum_batch_host(dg, n, stride=L, seg_len=L),
        "wrap": lambda: eng.tcp_wrap_batch_host(dg, m, n, stride=L, dgram_len=L),
        "wrap_const7": lambda: eng.tcp_wrap_batch_host(dg7, m, n, stride=L, dgram_len=L),
        "wrap_slice": lambda: eng.tcp_wrap_batch_host(dg, big[:n], n, stride=L, dgram_len=L),
        "wrap_x5": lambda: five(dg, m),
        "wrap_const7_slice_x5": lambda: five(dg7, big[:n]),
        "headers": lambda: eng.tcp_wrap_headers_host(pl, m, n, stride=P, payload_len=P),
        "copy": lambda: (d.copy_(dgt, non_blocking=False), torch.cuda.synchronize()),
    }
    # the two wrap forms agree (headers written in place == headers apart)
    cases["wrap"]()
    h = cases["headers"]()
    assert (dg.reshape(n, L)[:, :40].reshape(-1) == np.asarray(h).reshape(-1)).all()
    if args.cases:
        cases = {k: cases[k] for k in args.cases.split(",")}
    ts = {k: [] for k in cases}
    for r in range(args.rounds):
        for k in (list(cases) if r % 2 == 0 else list(cases)[::-1]):
            cases[k]()
            t0 = time.perf_counter()
            cases[k]()
            ts[k].append(time.perf_counter() - t0)
    for k, v in ts.items():
        med = statistics.median(v) / (5 if k.endswith("_x5") else 1)
        print(json.dumps({"case": k, "ms_median": round(med * 1e3, 3), "ms_min": round(min(v) * 1e3 / (5 if k.endswith("_x5") else 1), 3),
                          "GB_s": round(n * L / med / 1e9, 2), "slots": args.slots, "slot_mb": args.slot_mb,
                          "extra_engines": args.extra_engines, "extra_streams": args.extra_streams}),
              flush=True)


if __name__ == "__main__":
    main()
