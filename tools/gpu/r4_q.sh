#!/bin/bash
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_q}; mkdir -p $O
timeout -k 10 300 tools/probe/mix_probe > $O/mix_probe.jsonl 2> $O/mix_probe.err
