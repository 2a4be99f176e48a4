#!/bin/bash
# Round 6: the tick server with 1 / 2 / 4 staggered polling waves — the
# host-path tests, then the per-tick A/B against the previous build
# (tools/probe/libicsum_r6base.so), one context per process, back to back
# and 30 us apart.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6poll}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_zc.py tests/test_gpu_host.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
L=tcpip_network_protocol_stack_amd/libicsum.so
export TICK_OPS=verify,checksum,wrap TICK_SIZES=1,16 TICK_CALLS=300 TICK_MEM=pinned
for gap in 0 30; do
  for rep in 1 2; do
    for v in tools/probe/libicsum_r6base.so@tick_server=20000 $L@tick_server=20000 $L@tick_server=20000,srv_pollers=2 $L@tick_server=20000,srv_pollers=4; do
      TICK_GAP_US=$gap timeout -k 10 200 tools/probe/tick_latency "$v" >> $O/tick.jsonl 2>> $O/tick.err
    done
  done
done
