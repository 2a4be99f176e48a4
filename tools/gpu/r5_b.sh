#!/bin/bash
# k_stream first look: the tile tests (both forms), the bounds build over
# them, then the stream / tile A/B on the VERDICT r4 shapes.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r5b}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tile.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_tile.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_bounds.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_bounds.log 2>&1
timeout -k 10 600 python3 tools/ab_stream.py > $O/ab_stream.jsonl 2> $O/ab_stream.err
