#!/bin/bash
# Round-2 second GPU call: GPU tests (new host-path, multi-rank, threaded
# unwrap cases), counter passes for configs 2 and 3, the PATCH sequence trace.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2b; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 120 tcpip_network_protocol_stack_amd/csrc/host/build/host_gpu_test > $O/host_gpu_test.log 2>&1
tools/gpu/pmc_rows.sh $O/pmc
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$GRAFT_REPO_ROOT/$O/patch_seq" -o run -- python3 "$GRAFT_REPO_ROOT/tools/patch_seq.py" \
   > "$GRAFT_REPO_ROOT/$O/patch_seq_traced.log" 2>&1)
timeout -k 10 120 python3 tools/patch_seq.py > $O/patch_seq.json 2>&1
