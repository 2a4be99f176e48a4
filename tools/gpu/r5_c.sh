#!/bin/bash
# tile tests, then the stream / tile A/B on the VERDICT r4 shapes (reduced
# variant set) and one counter pass (SQ) over the 1 M x 770 B rows.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r5x}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tile.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_tile.log 2>&1
timeout -k 10 600 python3 tools/ab_stream.py tx256k,tx1m,u770_256k,u770_1m ${2:-tile,stream,stream_T256} > $O/ab_stream.jsonl 2> $O/ab_stream.err
export TMPDIR=/tmp AB_LIGHT=1
OUT=$(realpath -m $O)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d "$OUT/g1" -o pmc -- \
    python3 tools/ab_stream.py u770_1m tile,stream checksum > "$OUT/g1.log" 2>&1
python3 tools/pmc_kernels.py r5x $OUT/g1 > $OUT/pmc_summary.jsonl
