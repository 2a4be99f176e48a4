#!/usr/bin/env python3
"""Dev tool: does PATCH's cost sit in the PATCH launch or in the launch after
it?  BASELINE config 2 (64 Ki x 1500 B IPv4 datagrams, 6 rotated copies) as
three back-to-back sequences of ics_ipv4_tcp_batch launches:
  A  60 x COMPUTE            B  60 x PATCH            C  60 x (PATCH, COMPUTE)
Run under `rocprofv3 --kernel-trace`: the trace's per-dispatch durations, in
launch order, split by phase (A: 60, B: 60, C: 120 alternating) give COMPUTE
after COMPUTE, PATCH after PATCH, PATCH after COMPUTE and COMPUTE after PATCH.
Without the tracer it prints the HIP-event time of each phase."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from tcpip_network_protocol_stack_amd.engine import Engine  # noqa: E402


def main():
    eng = Engine(0)
    dev = torch.device("cuda", 0)
    n, L, seed, R = 1 << 16, 1500, 0x10710002, 6
    bufs = []
    for r in range(R):
        d = eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L)
        eng.ipv4_tcp_headers(d, n, L, L, seed, index0=r * n)
        bufs.append(d)
    ip = torch.empty(n, dtype=torch.int16, device=dev)
    tcp = torch.empty(n, dtype=torch.int16, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)

    def call(i, mode):
        eng.ipv4_tcp_batch(bufs[i % R], mode, n=n, stride=L, dgram_len=L, ip_ck=ip, tcp_ck=tcp, status=st)

    t0 = time.perf_counter()  # settle the clocks on the same work (untimed)
    while time.perf_counter() - t0 < 0.15:
        for i in range(8):
            call(i, 0)
        torch.cuda.synchronize()
    phases = {"A_compute": [0] * 60, "B_patch": [2] * 60, "C_patch_compute": [2, 0] * 60}
    out = {}
    for name, modes in phases.items():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for i, m in enumerate(modes):
            call(i, m)
        b.record()
        torch.cuda.synchronize()
        out[name] = round(a.elapsed_time(b) * 1e3 / len(modes), 2)
    print(json.dumps({"us_per_launch": out}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
