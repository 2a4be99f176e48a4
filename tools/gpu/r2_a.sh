#!/bin/bash
# Round-2 first GPU call: GPU tests, the bench line (N=1 and a one-card N=2
# rehearsal through bench.py's own launcher), the NS kernel trace, and the
# counter passes for configs 2 and 3.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench_ns.json 2> $O/bench_ns.err
ICSUM_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --no-pmc --steps 20 > $O/bench_n2_gloo.json 2> $O/bench_n2.err
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$GRAFT_REPO_ROOT/$O/ns_trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-pmc --cpu-seconds 0 \
   > "$GRAFT_REPO_ROOT/$O/bench_ns_under_rocprof.json" 2>&1)
tools/gpu/pmc_rows.sh $O/pmc
