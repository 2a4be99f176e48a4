#!/bin/bash
# Round 6: k_span builds A/B (tools/probe/<lib>, comma list $1) — the tile /
# any-base / offsets tests under the in-tree build, then tools/ab_stream.py
# (variant auto) under each build twice, alternating; the in-tree library is
# restored on every exit.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${2:-r6spanab}; mkdir -p $O
L=tcpip_network_protocol_stack_amd/libicsum.so
KEEP=$(mktemp /tmp/libicsum_keep.XXXXXX)
cp $L $KEEP
trap 'cp "$KEEP" "$L"; rm -f "$KEEP"' EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_tile.py tests/test_gpu_base_align.py tests/test_gpu_offsets_4g.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
for rep in 1 2; do
  for lib in ${1//,/ }; do
    cp tools/probe/$lib $L
    timeout -k 10 300 python3 tools/ab_stream.py ${3:-tx1m,tx256k,u770_1m} auto ${4:-checksum,verify,wrap_apart} | sed "s/^{/{\"lib\": \"$lib\", \"rep\": $rep, /" >> $O/ab.jsonl
  done
done
