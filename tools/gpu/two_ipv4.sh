#!/bin/bash
# Two-class fused IPv4 launch: every GPU test, then the receive-mix sweep.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-two3}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
AB_LANE1=1 timeout -k 10 300 python3 -u tools/ab_ipv4_mix.py 1.0,0.75,0.5,0.3125,0.25,0.0 > $O/ab_mix.jsonl 2> $O/ab_mix.err
