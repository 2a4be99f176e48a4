#!/bin/bash
# round 5: runtime span size — the tile tests, then the span-size sweep
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5n; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tile.py tests/test_gpu_bounds.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
timeout -k 10 700 python3 tools/ab_stream.py c4_128k,tx1m,u770_1m auto,per_segment,S2,S4,S8,S16,S32,S63 checksum,verify,wrap,wrap_apart > $O/ab.jsonl 2> $O/ab.err
