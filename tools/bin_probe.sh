# rocprofv3 kernel traces of tools/bin_probe.py per dispatch variant -> gpurun_out/binprobe/<tag>/
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/binprobe
mkdir -p $R
cd /tmp
run() {  # tag kind env...
  tag=$1; kind=$2; shift 2
  ( export "$@"; timeout -k 10 200 rocprofv3 --kernel-trace -d $R/$tag -o run -- python3 $GRAFT_REPO_ROOT/tools/bin_probe.py $kind 5 > $R/$tag.log 2>&1 )
}
run mixed_nobin mixed ICSUM_FORCE=bin=0
run mixed_bin mixed ICSUM_FORCE=bin=1
run bimodal_bin bimodal ICSUM_FORCE=bin=1
run bimodal_nobin bimodal ICSUM_FORCE=bin=0
run long_nobin long ICSUM_FORCE=bin=0
run long_bin long ICSUM_FORCE=bin=1
