#!/bin/bash
# Several builds of libicsum.so in one box: the in-tree one ("base"), then
# each tools/probe/<lib> of $1 (comma-separated) copied over it in turn; the
# tile tests and tools/ab_stream.py rows ($2, variant auto, ops $3) under
# each.  Output: gpurun_out/$4/{pytest,ab}_<name>.*
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$4; mkdir -p $O
cp tcpip_network_protocol_stack_amd/libicsum.so $O/../libicsum_base_copy.so
run() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_tile.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_$1.log 2>&1
  timeout -k 10 300 python3 tools/ab_stream.py $2 auto $3 > $O/ab_$1.jsonl 2> $O/ab_$1.err
}
run base "$2" "$3"
for lib in ${1//,/ }; do
  cp tools/probe/$lib tcpip_network_protocol_stack_amd/libicsum.so
  run "${lib%.so}" "$2" "$3"
done
rm -f $O/../libicsum_base_copy.so
