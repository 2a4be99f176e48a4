#!/bin/bash
# Round-2: device-side wrap — GPU tests, host_gpu_test, wrap rates, kernel trace.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_wrap.py tests/test_gpu_host.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_wrap.log 2>&1
timeout -k 10 200 python3 tools/bench_configs.py --only wrap,ipv4 > $O/wrap_rates.jsonl 2> $O/wrap_rates.err
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$GRAFT_REPO_ROOT/$O/wrap_trace" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --only wrap \
   > "$GRAFT_REPO_ROOT/$O/wrap_under_trace.jsonl" 2>&1)
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_all.log 2>&1
