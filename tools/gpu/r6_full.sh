#!/bin/bash
# Driver-equivalent check on the round-6 code: GPU tests, smoke, bench N=1
# (PMC, CPU baseline, host-inclusive) and its rocprof kernel stats, the
# one-card N=2 rehearsal, then the bench_configs rows.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6full}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$GRAFT_REPO_ROOT/$O/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-pmc --no-host --cpu-seconds 0 --steps 20 \
   > "$GRAFT_REPO_ROOT/$O/bench_under_rocprof.json" 2>&1)
timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 3 --no-pmc --cpu-seconds 0 > $O/bench_n2.json 2> $O/bench_n2.err
timeout -k 10 900 python3 tools/bench_configs.py --only ${2:-ns,ipv4,ns64k,tcp64,mixed,bimodal,jumbo,jumbo_all,host,router,wrap,streams,batchv,stack,rxmix} > $O/configs.jsonl 2> $O/configs.err
