#!/bin/bash
# Round 3: config-3 batchv variants, then the whole-sector store probes with counters.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3b}; mkdir -p $O
timeout -k 10 180 python3 tools/ab_batchv.py > $O/ab_batchv.jsonl 2> $O/ab_batchv.err
bash tools/gpu/r3_probe.sh ${1:-r3b}/probe
