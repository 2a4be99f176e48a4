#!/bin/bash
# Round 4: VALU / LDS counters of the stack rows' kernels (is k_tile ALU-bound?).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$(realpath -m gpurun_out/${1:-r4_i}); mkdir -p $O
BC="tools/bench_configs.py --settle-ms 0 --rounds 1 --iters 3 --only stack"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU \
  --output-format csv -d $O/valu -o pmc -- python3 $BC > $O/valu.log 2>&1
