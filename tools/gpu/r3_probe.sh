#!/bin/bash
# Round 3, verdict item 4: whole-sector stores instead of masked field stores
# (PATCH: ipv4_probe p9, router: router_probe sec), timed interleaved in one
# process, then memory-side write counters per variant, one rocprofv3 --pmc
# pass per counter group (no tracing domains).  Usage: r3_probe.sh OUTDIR
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=$(realpath -m "gpurun_out/${1:-r3probe}"); mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 120 tools/probe/ipv4_probe > "$O/ipv4_probe.jsonl" 2> "$O/ipv4_probe.err"
timeout -k 10 120 tools/probe/router_probe > "$O/router_probe.jsonl" 2> "$O/router_probe.err"
WR="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum"
ST="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum"
RD="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
for g in WR ST RD; do
  for p in ipv4_probe router_probe; do
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc ${!g} --output-format csv -d "$O/${p}_$g" -o pmc -- \
       "$GRAFT_REPO_ROOT/tools/probe/$p" > "$O/${p}_$g.log" 2>&1)
  done
done
# the shipped kernels' rows (the current two-lane router, PATCH / COMPUTE)
BC="tools/bench_configs.py --settle-ms 0 --rounds 1 --iters 2"
for g in WR ST RD; do
  timeout -s KILL 200 rocprofv3 --pmc ${!g} --output-format csv -d "$O/router_$g" -o pmc -- python3 $BC --only router \
    > "$O/router_$g.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc ${!g} --output-format csv -d "$O/ipv4_patch_$g" -o pmc -- python3 $BC --only ipv4 --modes patch \
    > "$O/ipv4_patch_$g.log" 2>&1
done
timeout -k 10 60 rocprofv3 --list-avail > "$O/list_avail.txt" 2>&1 || true
