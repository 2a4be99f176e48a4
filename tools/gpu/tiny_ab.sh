#!/bin/bash
# Tiny-segment kernel in the AUTO dispatch: every GPU test, the tiny A/B, and
# the plan-cached vs uncached dispatch on the mixes (outputs compared).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-tiny2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python3 -u tools/ab_tiny.py > $O/ab_tiny.jsonl 2> $O/ab_tiny.err
timeout -k 10 300 python3 -u tools/ab_lastbin.py --var bin --caps=-1,1 --workloads ack,bimodal,config4,mss > $O/ab_cache.jsonl 2> $O/ab_cache.err
