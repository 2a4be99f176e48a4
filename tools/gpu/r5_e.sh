#!/bin/bash
# k_span register sets A/B: the four tile shapes, then the stack rows under
# each setting
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r5x}; mkdir -p $O
timeout -k 10 600 python3 tools/ab_stream.py tx256k,tx1m,u770_256k,u770_1m span,span2 > $O/ab_stream.jsonl 2> $O/ab_stream.err
timeout -k 10 300 python3 tools/bench_configs.py --only stack > $O/stack_span3.jsonl 2> $O/stack3.err
ICSUM_FORCE=span_sets=2 timeout -k 10 300 python3 tools/bench_configs.py --only stack > $O/stack_span2.jsonl 2> $O/stack2.err
