#!/bin/bash
# tile tests, stream / tile A/B (reduced variant set), k_stream stamps
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r5x}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tile.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_tile.log 2>&1
timeout -k 10 120 tools/probe/stream_stamps > $O/stamps.jsonl 2>&1
timeout -k 10 600 python3 tools/ab_stream.py tx256k,tx1m,u770_256k,u770_1m ${2:-tile,stream,stream_T256,span} > $O/ab_stream.jsonl 2> $O/ab_stream.err
timeout -k 10 120 tools/probe/verify_stamps > $O/verify_stamps.jsonl 2>&1
