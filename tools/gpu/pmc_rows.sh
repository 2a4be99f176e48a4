#!/bin/bash
# Counter passes (one rocprofv3 --pmc run per counter group, no tracing domains)
# for the kernels below the NS roofline: k_ipv4_tcp in COMPUTE / PATCH / VERIFY
# on BASELINE config 2 and k_checksum_dense on config 3, plus the kernel-trace
# stats of the same rows.  Usage: tools/gpu/pmc_rows.sh OUTDIR
set -euo pipefail
OUT=$(realpath -m "$1"); mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
BC="tools/bench_configs.py --settle-ms 0 --rounds 1 --iters 2"
for row in compute patch verify; do
  for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" \
             "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
    tag=$(echo "$grp" | cut -d' ' -f1)
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d "$OUT/ipv4_${row}_$tag" -o pmc -- \
      python3 $BC --only ipv4 --modes $row > "$OUT/ipv4_${row}_$tag.log" 2>&1
  done
done
for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  tag=$(echo "$grp" | cut -d' ' -f1)
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d "$OUT/tcp64_$tag" -o pmc -- \
    python3 $BC --only tcp64 > "$OUT/tcp64_$tag.log" 2>&1
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 tools/bench_configs.py --only ipv4,tcp64 > "$OUT/trace.log" 2>&1
