#!/bin/bash
# Round 4: the tile launch across 2^31 / 2^32 byte offsets and under the bounds-checked build.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_k}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_bounds.py tests/test_gpu_offsets_4g.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --durations=5 > $O/pytest.log 2>&1
