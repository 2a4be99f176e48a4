#!/bin/bash
# round 5: k_span on every tile operation — the tile tests, then the A/B
set -o pipefail
O=gpurun_out/r5k; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tile.py -x -q --timeout 120 --timeout-method thread > $O/pytest_tile.log 2>&1 &&
timeout -k 10 500 python3 tools/ab_stream.py tx256k,tx1m,u770_1m tile,span checksum,wrap_apart,wrap,verify,patch > $O/ab.jsonl 2> $O/ab.err
