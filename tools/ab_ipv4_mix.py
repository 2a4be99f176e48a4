#!/usr/bin/env python3
"""Dev measurement: the fused IPv4/TCP kernel (VERIFY / COMPUTE) over a
received-traffic mix — raw datagrams back to back (offsets), half of them
40-byte pure ACKs and half 1500-byte data segments — at the default geometry
(16-lane groups for offsets batches) and at forced ones, beside the plain
checksum of the same bytes (binned AUTO, and single launches at the forced
geometries) and the all-MTU batch.  Argument: comma-separated ACK shares."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tcpip_network_protocol_stack_amd.engine import Engine  # noqa: E402
from _force import engine, geometry  # noqa: E402

PEAK = 8.0e12


def engine_with(lps, unroll, mode):
    return engine(**geometry(lps, unroll, mode))


def timed(fn, iters=20, rounds=5):
    st = torch.cuda.current_stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.1:
        fn()
        torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(iters):
            fn()
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 1e3 / iters)
    return float(np.median(ts))


def batch(eng, n, ack_frac, seed):
    rng = np.random.default_rng(seed)
    lens = np.where(rng.random(n) < ack_frac, 40, 1500).astype(np.uint64)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    s = off[:-1].astype(np.int64)
    buf[s] = 0x45
    buf[s + 1] = 0
    buf[s + 2] = (lens >> 8).astype(np.uint8)
    buf[s + 3] = (lens & 255).astype(np.uint8)
    buf[s + 6] = 0x40
    buf[s + 7] = 0
    buf[s + 8] = 64
    buf[s + 9] = 6
    buf[s + 32] = 0x50  # TCP data offset 5
    d = torch.from_numpy(buf).cuda()
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    eng.ipv4_tcp_batch(d, 2, n=n, offsets=doff)  # PATCH: valid checksums
    return d, doff, int(off[-1])


def main():
    eng = Engine(0)
    forced = {f"{l}x{u}m{m}": engine_with(l, u, m) for l, u, m in ((4, 2, 2), (8, 2, 2), (8, 4, 3), (8, 8, 3), (16, 4, 3), (16, 8, 3), (32, 8, 3))}
    if os.environ.get("AB_LANE1"):  # one lane per datagram (mode 4: the IPv4 kernel's default-policy lane1 shape)
        forced = {k: forced[k] for k in ("4x2m2", "8x8m3")}
        forced.update({"1x4m4": engine_with(1, 4, 4)})
    fracs = [float(a) for a in sys.argv[1].split(",")] if len(sys.argv) > 1 else (0.5, 0.0)
    for ack_frac in fracs:
        n = 1 << 20
        d, doff, nbytes = batch(eng, n, ack_frac, 7)
        ip = torch.empty(n, dtype=torch.int16, device="cuda")
        tcp = torch.empty(n, dtype=torch.int16, device="cuda")
        st = torch.empty(n, dtype=torch.uint8, device="cuda")
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        rows = {"plain_auto": lambda: eng.checksum_batch(d, offsets=doff, out=out),
                "verify_default": lambda: eng.ipv4_tcp_batch(d, 1, n=n, offsets=doff, ip_ck=ip, tcp_ck=tcp, status=st),
                "compute_default": lambda: eng.ipv4_tcp_batch(d, 0, n=n, offsets=doff, ip_ck=ip, tcp_ck=tcp,
                                                              status=st)}
        for k, e in forced.items():
            rows[f"verify_{k}"] = (lambda e: lambda: e.ipv4_tcp_batch(d, 1, n=n, offsets=doff, ip_ck=ip, tcp_ck=tcp,
                                                                     status=st))(e)
            rows[f"plain_{k}"] = (lambda e: lambda: e.checksum_batch(d, offsets=doff, out=out))(e)
        for k, fn in rows.items():
            t = timed(fn)
            print(json.dumps({"ack_frac": ack_frac, "n": n, "bytes": nbytes, "case": k, "us": round(t * 1e6, 2),
                              "frac_hbm_peak": round(nbytes / t / PEAK, 4)}), flush=True)
        eng.ipv4_tcp_batch(d, 1, n=n, offsets=doff, status=st)
        torch.cuda.synchronize()
        assert (st.cpu().numpy() & 0x03 == 0x03).all()
        del d


if __name__ == "__main__":
    main()
