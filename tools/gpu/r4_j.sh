#!/bin/bash
# Round 4: k_tile with one wave scan per window — tile parity, then the
# previous build vs this one on the stack rows and the tile-size sweep rows.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_j}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tile.py tests/test_gpu_stack_tick.py tests/test_gpu_bounds.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
bash tools/probe/ab_libs.sh stack 3 tools/probe/libicsum_pretile.so tools/probe/libicsum_tposed.so > $O/ab.jsonl 2> $O/ab.err
