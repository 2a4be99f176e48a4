#!/bin/bash
# Round 3, first GPU pass: the whole GPU suite (new: >4 GiB offsets, config 5
# in 8 engine processes, config 4 byte-balanced shards), then bench.py at N=1
# and the one-card gloo rehearsals of N=2 and N=4 (NS weak + config-5 strong).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3a}; mkdir -p $O
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider --durations=25 > $O/pytest.log 2>&1
timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 > $O/bench_n1.json 2> $O/bench_n1.err
timeout -k 10 240 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 > $O/bench_n2.json 2> $O/bench_n2.err
timeout -k 10 300 python3 bench.py --gpus 4 --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 > $O/bench_n4.json 2> $O/bench_n4.err
timeout -k 10 300 python3 tools/bench_configs.py --only ipv4,ns64k,tcp64,streams,batchv > $O/configs_short.jsonl 2> $O/configs_short.err
