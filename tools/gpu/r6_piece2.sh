#!/bin/bash
# Round 6: k_piece with its first pass requested before the points' chunk
# loads (no dependent offsets -> point-load chain ahead of the stream) —
# the tile / any-base tests, then the A/B against k_span.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6piece2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tile.py tests/test_gpu_base_align.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
timeout -k 10 500 python3 tools/ab_stream.py ${2:-tx1m,u770_1m,tx256k} ${3:-S32,piece,P8192,P12288,K12P12288,K12P16384} ${4:-checksum,verify,wrap_apart} > $O/ab.jsonl 2> $O/ab.err
