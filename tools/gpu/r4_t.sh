#!/bin/bash
# Round 4: two-class COMPUTE / VERIFY verdicts computed at block end: parity, then A/B.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_t}; mkdir -p $O
# timeout -k 10 600 python -u -m pytest tests/test_gpu_twoclass.py tests/test_gpu_bounds.py tests/test_gpu_offsets_4g.py tests/test_gpu_stack_tick.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
bash tools/probe/ab_libs.sh stack 4 tools/probe/libicsum_base5.so tools/probe/libicsum_vstash.so tools/probe/libicsum_vraw.so > $O/ab.jsonl 2> $O/ab.err
