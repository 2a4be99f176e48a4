#!/bin/bash
# Round 4: the tile launches — parity first, then the A/B.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_tile}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tile.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_tile.log 2>&1
timeout -k 10 300 python3 tools/ab_tile.py 262144 > $O/abtile256k.jsonl 2> $O/abtile256k.err
timeout -k 10 400 python3 tools/ab_tile.py 1048576 > $O/abtile1m.jsonl 2> $O/abtile1m.err
