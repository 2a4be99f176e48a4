#!/bin/bash
# Round 6: k_piece parity (tile + any-base suites, bounds build included),
# then the span / piece A/B rows.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6piece}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tile.py tests/test_gpu_base_align.py tests/test_gpu_bounds.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
timeout -k 10 600 python3 tools/ab_stream.py ${2:-tx256k,tx1m,u770_1m} ${3:-span,piece,P3072,P4096,P8192,P12288} ${4:-checksum,wrap_apart,verify} > $O/ab.jsonl 2> $O/ab.err
