#!/bin/bash
# Round 4: the two-class VERIFY with its mode as a compile-time constant — parity, A/B.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_n}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_twoclass.py tests/test_gpu_stack_tick.py tests/test_gpu_offsets_4g.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
bash tools/probe/ab_libs.sh stack,rxmix 3 tools/probe/libicsum_tposed.so tools/probe/libicsum_modet.so > $O/ab.jsonl 2> $O/ab.err
