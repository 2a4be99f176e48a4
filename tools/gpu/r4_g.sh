#!/bin/bash
# Round 4: tile size from the plan's mean length — its tests, the stack rows
# (HIP events) and their kernel trace, the dispatch A/B at 256 Ki.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_g}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tile.py tests/test_gpu_stack_tick.py tests/test_gpu_wrap.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
timeout -k 10 300 python3 tools/bench_configs.py --only stack > $O/stack_rows.jsonl 2> $O/stack_rows.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o stack -- python3 tools/bench_configs.py --only stack > $O/stack_traced.jsonl 2> $O/trace.err
timeout -k 10 600 python3 tools/ab_dispatch.py 262144 > $O/dispatch.jsonl 2> $O/dispatch.err
