#!/bin/bash
# Round 4: the whole GPU suite on the new dispatch and the in-kernel completion,
# the per-tick A/B against the previous build (k_host_flag), the dispatch A/B
# and the stack rows.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_c}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider --durations=15 > $O/pytest.log 2>&1
TICK_OPS=checksum,verify,wrap TICK_MEM=pinned TICK_SIZES=1,16,256 timeout -k 10 300 tools/probe/tick_latency tools/probe/libicsum_head.so tcpip_network_protocol_stack_amd/libicsum.so > $O/tick_ab.jsonl 2> $O/tick_ab.err
timeout -k 10 600 python3 tools/ab_dispatch.py 262144,1048576 > $O/dispatch.jsonl 2> $O/dispatch.err
timeout -k 10 300 python3 tools/bench_configs.py --only stack > $O/stack_rows.jsonl 2> $O/stack_rows.err
