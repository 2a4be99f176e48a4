#!/bin/bash
# Round 6: the any-base module, then the whole GPU suite (one process each),
# then the per-tick A/B (k_tick vs the grid launches, one process).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6tests}; mkdir -p $O
L=tcpip_network_protocol_stack_amd/libicsum.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_base_align.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_align.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
TICK_OPS=verify,verify_off,checksum_off TICK_SIZES=1,16 TICK_MEM=pinned timeout -k 10 300 \
  tools/probe/tick_latency $L $L@tick_inline=0 > $O/tick_ab.jsonl 2> $O/tick_ab.err
