#!/bin/bash
# Round 4: plain two-class checksum with its sums staged in LDS: parity, then A/B.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_s}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_twoclass.py tests/test_gpu_bounds.py tests/test_gpu_offsets_4g.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
bash tools/probe/ab_libs.sh bimodal 3 tools/probe/libicsum_base4.so tools/probe/libicsum_csumlds.so > $O/ab.jsonl 2> $O/ab.err
