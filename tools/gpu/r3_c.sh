#!/bin/bash
# Round 3: config-3 multi-batch variants (SEGS 4/8, XCD-aware vs hardware
# block order) and the PATCH store-shape probe with the p9 equality check.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3c}; mkdir -p $O
timeout -k 10 180 python3 tools/ab_batchv.py > $O/ab_batchv.jsonl 2> $O/ab_batchv.err
timeout -k 10 120 tools/probe/ipv4_probe > $O/ipv4_probe.jsonl 2> $O/ipv4_probe.err
