#!/bin/bash
# Round 4: fused IPv4 two-class variants on the stack rows (VGPRs / unroll).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_d}; mkdir -p $O
bash tools/probe/ab_libs.sh stack 3 tools/probe/libicsum_base.so tools/probe/libicsum_u6.so tools/probe/libicsum_u6o8.so > $O/ab.jsonl 2> $O/ab.err
