#!/bin/bash
# Round 6: the resident tick server — its tests, then the per-tick A/B
# (launched k_tick / grid launches vs the server), one context per process.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6srv}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_zc.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
TICK_OPS=verify,verify_off,checksum,checksum_off,wrap bash tools/gpu/r6_tick_ab.sh ${1:-r6srv} "" tick_server=20000
