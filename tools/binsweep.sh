# binned dispatch settings vs the single-geometry dispatch (tools/bench_configs.py)
# BINSWEEP_FORCE: space-separated settings, each an ICSUM_FORCE value (key=value,...)
mkdir -p gpurun_out && export TMPDIR=/tmp
for cfg in ${BINSWEEP_FORCE:-bin_blocks=2048 bin_blocks=8192}; do
  ( export ICSUM_FORCE=$cfg; timeout -k 10 200 python tools/bench_configs.py --only ${BINSWEEP_ONLY:-mixed,bimodal} --iters 10 > gpurun_out/binsweep_${cfg//[=,]/_}.jsonl 2>&1 ) || exit 1
done
