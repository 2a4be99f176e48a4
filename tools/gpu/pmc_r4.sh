#!/bin/bash
# Round 4 counters: the stack-tick rows (k_ipv4_twoclass VERIFY, k_tcp_wrap,
# k_tile headers apart) and the router rows (k_router_ttl, k_router_hdrs).
# One rocprofv3 --pmc run per counter group (FETCH_SIZE and WRITE_SIZE in
# separate passes: 3 + 2 TCC counters exceed one pass), no tracing domains;
# then the kernel-trace stats of the same rows.  Usage: tools/gpu/pmc_r4.sh OUTDIR
set -euo pipefail
OUT=$(realpath -m "$1"); mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
BC="tools/bench_configs.py --settle-ms 0 --rounds 1 --iters 3"
for rows in stack router; do
  for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"; do
    tag=$(echo "$grp" | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/${rows}_$tag" -o pmc -- \
      python3 $BC --only $rows > "$OUT/${rows}_$tag.log" 2>&1
  done
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 tools/bench_configs.py --only stack,router > "$OUT/trace.log" 2>&1
