#!/bin/bash
# Flat dispatch of offsets batches: GPU parity tests, then A/B against the
# current AUTO dispatch (outputs compared) and over the wave count.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-flat}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py -x -q --timeout 120 --timeout-method thread > $O/pytest_flat.log 2>&1
timeout -k 10 300 python3 -u tools/ab_lastbin.py --var ICSUM_FLAT --caps 0,1 --workloads config4,bimodal,mss,ack,long2m > $O/ab_flat.jsonl 2> $O/ab_flat.err
ICSUM_FLAT=1 timeout -k 10 300 python3 -u tools/ab_lastbin.py --var ICSUM_FLAT_WAVES --caps 4096,16384,49152,131072 --workloads config4,long2m,mss > $O/ab_flat_waves.jsonl 2> $O/ab_flat_waves.err
