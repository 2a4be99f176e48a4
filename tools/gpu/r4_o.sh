#!/bin/bash
# Round 4: k_tile with a per-lane prefix only (26.6 KB of LDS; the checksum at 5 waves / SIMD):
# tile parity, then the previous build vs this one (stack rows; tile-size sweep rows per build).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4_o}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tile.py tests/test_gpu_stack_tick.py tests/test_gpu_bounds.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
bash tools/probe/ab_libs.sh stack 2 tools/probe/libicsum_base2.so tools/probe/libicsum_tlds.so > $O/ab.jsonl 2> $O/ab.err
L=tcpip_network_protocol_stack_amd/libicsum.so
cp $L /tmp/keep.so
for r in 1 2; do
  for v in tools/probe/libicsum_base2.so tools/probe/libicsum_tlds.so; do
    cp $v $L
    timeout -k 10 300 python3 tools/ab_tile_T.py 262144,1048576 128,192,256 | sed "s|^{|{\"build\": \"$(basename $v)\", |" >> $O/tileT.jsonl
  done
done
cp /tmp/keep.so $L
