#!/bin/bash
# Stack rows with and without a resident tick-server block elsewhere on the
# card (a second engine): does the idle-queue cost of a single call change?
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6warm}; mkdir -p $O
for v in -1 0 5000000 -1 5000000; do
  timeout -k 10 240 python3 tools/bench_configs.py --only stack --warm-server $v > $O/stack_$v.jsonl 2> $O/stack_$v.err
  mv $O/stack_$v.jsonl $O/stack_${v}_$(date +%s%N).jsonl
done
