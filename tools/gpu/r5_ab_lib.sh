#!/bin/bash
# Several builds of libicsum.so in one box: the in-tree one ("base"), then
# each tools/probe/<lib> of $1 (comma-separated) copied over it in turn; the
# tile tests and tools/ab_stream.py rows ($2, variant auto, ops $3) under
# each.  Output: gpurun_out/$4/{pytest,ab}_<name>.*  The in-tree library is
# restored on every exit (a diagnostic build gives wrong results), and a
# variant whose tests fail does not stop the others.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$4; mkdir -p $O
L=tcpip_network_protocol_stack_amd/libicsum.so
KEEP=$(mktemp /tmp/libicsum_base.XXXXXX)
cp $L $KEEP
trap 'cp "$KEEP" "$L"; rm -f "$KEEP"' EXIT
run() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_tile.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_$1.log 2>&1 || echo "$1: tests failed (rc $?)" >> $O/failed.txt
  timeout -k 10 300 python3 tools/ab_stream.py $2 auto $3 > $O/ab_$1.jsonl 2> $O/ab_$1.err
}
run base "$2" "$3"
for lib in ${1//,/ }; do
  cp tools/probe/$lib $L
  run "${lib%.so}" "$2" "$3"
done
