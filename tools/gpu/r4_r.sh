#!/bin/bash
# Round 4: two-class VERIFY outputs staged in LDS (coalesced rows): parity, the
# decomposition probe, then the previous build vs this one.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_r}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_twoclass.py tests/test_gpu_stack_tick.py tests/test_gpu_bounds.py tests/test_gpu_offsets_4g.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
timeout -k 10 300 tools/probe/mix_probe > $O/mix_probe.jsonl 2> $O/mix_probe.err
bash tools/probe/ab_libs.sh stack,rxmix 3 tools/probe/libicsum_base3.so tools/probe/libicsum_ldsout.so > $O/ab.jsonl 2> $O/ab.err
