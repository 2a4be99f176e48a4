#!/bin/bash
# Round 4: the changed GPU tests, the two-class residency / datagrams-per-wave
# sweep, the tile-size sweep, then the counter passes of the stack and router rows.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_f}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stack_tick.py tests/test_gpu_twoclass.py tests/test_gpu_parity.py tests/test_gpu_bounds.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
timeout -k 10 400 python3 tools/ab_twoclass_lds.py > $O/lds.jsonl 2> $O/lds.err
timeout -k 10 500 python3 tools/ab_tile_T.py > $O/tileT.jsonl 2> $O/tileT.err
bash tools/gpu/pmc_r4.sh $O/pmc
