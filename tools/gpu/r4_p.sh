#!/bin/bash
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_p}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_concurrency.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
