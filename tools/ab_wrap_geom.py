#!/usr/bin/env python3
"""Dev A/B: where the headers-apart wrap's time over the plain checksum goes.
1 M x 1000-byte payloads (the stack's MSS), interleaved rounds in one process:
the plain checksum of the payloads, ics_tcp_wrap_headers at the default
geometry and at forced geometries (ICSUM_LPS/UNROLL/MODE, read at ics_create),
and the in-place wrap of the 1040-byte datagrams."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tcpip_network_protocol_stack_amd.engine import TCP_MSG_DTYPE, Engine  # noqa: E402

GEOMS = [(16, 4), (16, 6), (16, 8), (32, 4), (64, 8)]


def engine_with(lps, unroll):
    os.environ.update(ICSUM_LPS=str(lps), ICSUM_UNROLL=str(unroll), ICSUM_MODE="3", ICSUM_NT="1")
    try:
        return Engine(0)
    finally:
        for k in ("ICSUM_LPS", "ICSUM_UNROLL", "ICSUM_MODE", "ICSUM_NT"):
            del os.environ[k]


def main():
    dev = torch.device("cuda", 0)
    base = Engine(0)
    forced = {f"{lps}x{u}": engine_with(lps, u) for lps, u in GEOMS}
    os.environ["ICSUM_WRAP_GROUP"] = "1"
    grp = Engine(0)  # the per-lane-group header pass (first round-2 kernel)
    del os.environ["ICSUM_WRAP_GROUP"]
    n, P, R = 1 << 20, 1000, 3
    rng = np.random.default_rng(6)
    m = np.zeros(n, dtype=TCP_MSG_DTYPE)
    for f in ("src", "dst", "seqno", "ackno"):
        m[f] = rng.integers(0, 2**32, n, dtype=np.uint64)
    m["flags"], m["ttl"] = 0x10, 128
    dm = torch.from_numpy(m.view(np.uint8).copy()).to(dev)
    ps = [base.fill_bytes(torch.empty(n * P, dtype=torch.uint8, device=dev), 0x1071, pos0=r * n * P)
          for r in range(R)]
    L = P + 40
    ds = [base.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), 0x1072, pos0=r * n * L)
          for r in range(R)]
    hd = torch.empty(n * 40, dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    cases = {
        "plain": lambda i: base.checksum_batch(ps[i % R], n=n, stride=P, seg_len=P, out=out),
        "apart": lambda i: base.tcp_wrap_headers(ps[i % R], dm, hd, n=n, stride=P, payload_len=P),
        "in_place": lambda i: base.tcp_wrap_batch(ds[i % R], dm, n=n, stride=L, dgram_len=L),
        "apart_group": lambda i: grp.tcp_wrap_headers(ps[i % R], dm, hd, n=n, stride=P, payload_len=P),
        "in_place_group": lambda i: grp.tcp_wrap_batch(ds[i % R], dm, n=n, stride=L, dgram_len=L),
    }
    for k, e in forced.items():
        cases[f"apart_{k}"] = (lambda e: lambda i: e.tcp_wrap_headers(ps[i % R], dm, hd, n=n, stride=P,
                                                                        payload_len=P))(e)
        cases[f"plain_{k}"] = (lambda e: lambda i: e.checksum_batch(ps[i % R], n=n, stride=P, seg_len=P,
                                                                     out=out))(e)
    res = {k: [] for k in cases}
    st = torch.cuda.current_stream()
    for rnd in range(5):
        for k, fn in cases.items():
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.04:
                for i in range(4):
                    fn(i)
                torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for i in range(20):
                fn(i)
            b.record(st)
            torch.cuda.synchronize()
            res[k].append(a.elapsed_time(b) * 1e3 / 20)
        print(f"round {rnd} done", file=sys.stderr, flush=True)
    for k, v in res.items():
        print(json.dumps({"case": k, "us": round(float(np.median(v)), 2), "min": round(float(min(v)), 2)}),
              flush=True)


if __name__ == "__main__":
    main()
