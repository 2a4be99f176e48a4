#!/bin/bash
# Round 4: where the stack-tick shapes lose time.
#   1. the stack rows + rxmix (1 M) under a kernel trace: per-kernel durations
#   2. the same rows' HIP-event figures (per call and back to back)
#   3. one PMC pass (FETCH_SIZE, WRITE_SIZE) over the stack rows
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_stack}; mkdir -p $O
timeout -k 10 240 python3 tools/bench_configs.py --only stack,rxmix --iters 20 > $O/rows.jsonl 2> $O/rows.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o stack -- \
  python3 tools/bench_configs.py --only stack --iters 20 > $O/rows_traced.jsonl 2> $O/trace.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --output-format csv -d $O/pmc -o stack -- \
  python3 tools/bench_configs.py --only stack --iters 4 --rounds 1 --settle-ms 0 > $O/rows_pmc.jsonl 2> $O/pmc.err
