#!/bin/bash
# round 5: k_span as the only tile launch — the GPU tests, then the A/B
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5l; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
timeout -k 10 500 python3 tools/ab_stream.py tx256k,tx1m,u770_1m span,per_segment checksum,wrap_apart,wrap,verify,patch > $O/ab.jsonl 2> $O/ab.err
