#!/bin/bash
# Round 4: persistent two-class VERIFY (next chunk's bounds prefetched): parity, then the sweep.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_m}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_twoclass.py tests/test_gpu_bounds.py tests/test_gpu_stack_tick.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
timeout -k 10 400 python3 tools/ab_twoclass_lds.py 262144,1048576 0 > $O/persist.jsonl 2> $O/persist.err
