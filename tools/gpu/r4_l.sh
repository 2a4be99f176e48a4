#!/bin/bash
# Round 4: the tile launch on batches of more than 2^32 segments.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_l}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_count_4g.py -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider --durations=8 > $O/pytest.log 2>&1
