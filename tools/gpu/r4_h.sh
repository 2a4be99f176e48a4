#!/bin/bash
# Round 4: the stack rows with the whole-tick rows (one and two streams).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_h}; mkdir -p $O
timeout -k 10 300 python3 tools/bench_configs.py --only stack > $O/stack_rows.jsonl 2> $O/stack_rows.err
