#!/bin/bash
# Counter passes (one rocprofv3 --pmc run per counter group, no tracing domains)
# for the receive-mix rows: k_ipv4_twoclass (block lists) on the rxmix rows
# and k_checksum_twoclass on the bimodal row, plus the kernel-trace stats of
# the same rows.  Usage: tools/gpu/pmc_rxmix.sh OUTDIR
set -euo pipefail
OUT=$(realpath -m "$1"); mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
BC="tools/bench_configs.py --settle-ms 0 --rounds 1 --iters 2 --only rxmix,bimodal"
for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  tag=$(echo "$grp" | cut -d' ' -f1)
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d "$OUT/rx_$tag" -o pmc -- \
    python3 $BC > "$OUT/rx_$tag.log" 2>&1
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 tools/bench_configs.py --only rxmix,bimodal > "$OUT/trace.log" 2>&1
