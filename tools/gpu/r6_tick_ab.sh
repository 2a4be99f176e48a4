#!/bin/bash
# Per-tick A/B, one engine context per process (several contexts in one
# process land their slot streams on shared hardware queues and differ by up
# to 6 us on identical code): each variant's process twice, alternating; the
# ops interleaved call by call inside each process.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6tick}; mkdir -p $O
L=tcpip_network_protocol_stack_amd/libicsum.so
export TICK_OPS=${TICK_OPS:-verify,verify_off,checksum,checksum_off} TICK_SIZES=${TICK_SIZES:-1,16} TICK_MEM=${TICK_MEM:-pinned} TICK_CALLS=${TICK_CALLS:-300}
shift || true
for rep in 1 2; do
  for v in "$@"; do
    timeout -k 10 200 tools/probe/tick_latency "$L${v:+@$v}" >> $O/tick.jsonl 2>> $O/tick.err
  done
done
