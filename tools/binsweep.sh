# binned dispatch settings vs the single-geometry dispatch (tools/bench_configs.py)
# BINSWEEP_ENVS: space-separated settings, each a comma-separated VAR=value list
mkdir -p gpurun_out && export TMPDIR=/tmp
for cfg in ${BINSWEEP_ENVS:-ICSUM_BIN_BLOCKS=2048 ICSUM_BIN_BLOCKS=8192}; do
  ( export ${cfg//,/ }; timeout -k 10 200 python tools/bench_configs.py --only ${BINSWEEP_ONLY:-mixed,bimodal} --iters 10 > gpurun_out/binsweep_${cfg//[=,]/_}.jsonl 2>&1 ) || exit 1
done
