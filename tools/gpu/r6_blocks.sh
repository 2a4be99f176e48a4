#!/bin/bash
# Round 6: the tick server over several resident blocks (srv_blocks) — the
# host-memory tests, then the per-tick A/B at 1..64 segments: launched,
# served by one block (<= 16 segments), served by four (<= 64).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6blk}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_zc.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
TICK_OPS=${TICK_OPS:-verify,checksum,wrap} TICK_SIZES=${TICK_SIZES:-1,16,64,128} \
  bash tools/gpu/r6_tick_ab.sh ${1:-r6blk} ${VARIANTS:-"" tick_server=20000,srv_blocks=1 tick_server=20000,srv_blocks=4 tick_server=20000,srv_blocks=8}
