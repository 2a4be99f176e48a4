#!/bin/bash
# Two-class launches as AUTO chooses them: every GPU test, the AUTO A/B and the ACK-share sweep.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-two5}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python3 -u tools/ab_lastbin.py --var ICSUM_TWOCLASS --caps 1,0 --workloads bimodal,ack,mss,config4 > $O/ab_auto.jsonl 2> $O/ab_auto.err
AB_LANE1=1 timeout -k 10 300 python3 -u tools/ab_ipv4_mix.py 0.875,0.75,0.625,0.5,0.4375,0.25 > $O/ab_mix.jsonl 2> $O/ab_mix.err
