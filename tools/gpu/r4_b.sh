#!/bin/bash
# Round 4: tile + router-headers parity, router rows, tile A/B.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_b}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tile.py tests/test_gpu_router_hdrs.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
timeout -k 10 300 python3 tools/bench_configs.py --only router > $O/router.jsonl 2> $O/router.err
timeout -k 10 300 python3 tools/ab_tile.py 262144 > $O/abtile256k.jsonl 2> $O/abtile256k.err
timeout -k 10 400 python3 tools/ab_tile.py 1048576 > $O/abtile1m.jsonl 2> $O/abtile1m.err
