mkdir -p gpurun_out && export TMPDIR=/tmp
for b in 1024 2048 8192 65536 4194304; do
  ICSUM_BIN_BLOCKS=$b timeout -k 10 200 python tools/bench_configs.py --only mixed,bimodal --iters 10 > gpurun_out/binsweep_$b.jsonl 2>&1 || exit 1
done
