#!/bin/bash
# Round 5, first run: GPU tests, bench N=1 (PMC, CPU baseline, host path),
# then bench.py's own launcher at N=2 and N=8 with every rank on this box's
# one card (the per-rank shard digests and device ids of VERDICT r4 item 1).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r5a}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 3 --no-pmc --cpu-seconds 0 > $O/bench_n2.json 2> $O/bench_n2.err
timeout -k 10 600 python3 bench.py --gpus 8 --steps 5 --warmup 2 --settle-ms 20 --config5-steps 3 --no-pmc --cpu-seconds 0 > $O/bench_n8.json 2> $O/bench_n8.err
