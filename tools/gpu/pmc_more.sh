#!/bin/bash
# Counter passes (one rocprofv3 --pmc run per counter group) for the NS,
# config-4 (mixed, AUTO dispatch) and config-5 shard (1 M x 9000 B) rows of
# tools/bench_configs.py, plus their kernel-trace stats.  Usage: pmc_more.sh OUTDIR
set -euo pipefail
OUT=$(realpath -m "$1"); mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
BC="tools/bench_configs.py --settle-ms 0 --rounds 1 --iters 2"
for row in ns mixed jumbo; do
  for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" \
             "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
    tag=$(echo "$grp" | cut -d' ' -f1)
    timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d "$OUT/${row}_$tag" -o pmc -- \
      python3 $BC --only $row > "$OUT/${row}_$tag.log" 2>&1
  done
done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 tools/bench_configs.py --only ns,mixed,jumbo > "$OUT/trace.log" 2>&1
