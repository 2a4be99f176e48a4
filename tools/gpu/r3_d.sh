#!/bin/bash
# Round 3: the multi-batch tests and the config-3 A/B after the scalar batch lookup.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3d}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batchv.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_batchv.log 2>&1
timeout -k 10 180 python3 tools/ab_batchv.py > $O/ab_batchv.jsonl 2> $O/ab_batchv.err
timeout -k 10 300 python3 tools/bench_configs.py --only batchv,ipv4,tcp64 > $O/configs_batchv.jsonl 2> $O/configs_batchv.err
