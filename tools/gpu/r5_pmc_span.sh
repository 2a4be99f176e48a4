#!/bin/bash
# SQ / memory counters (one rocprofv3 --pmc pass per group, no tracing
# domains) of k_span under the default dispatch on the transmit mix (256 Ki:
# the stack tick; 1 M) and 1 M x 770 B, checksum and headers-apart wrap
# (tools/ab_stream.py, a few calls per row).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$(realpath -m gpurun_out/${1:-r5pmc}); mkdir -p "$OUT"
export TMPDIR=/tmp AB_LIGHT=1
for row in tx256k tx1m u770_1m; do
  i=0; mkdir -p "$OUT/$row"
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
             "SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM" \
             FETCH_SIZE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/$row/g$i" -o pmc -- \
      python3 tools/ab_stream.py $row auto checksum,wrap_apart > "$OUT/$row/g$i.log" 2>&1
  done
  python3 tools/pmc_kernels.py $row $OUT/$row/g1 $OUT/$row/g2 $OUT/$row/g3 >> $OUT/summary.jsonl
done
