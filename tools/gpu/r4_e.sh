#!/bin/bash
# Round 4: two-class residency sweep (dynamic LDS cap) on the receive mix.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_e}; mkdir -p $O
timeout -k 10 400 python3 tools/ab_twoclass_lds.py > $O/lds.jsonl 2> $O/lds.err
