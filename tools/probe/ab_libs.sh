# dev: interleaved A/B of several builds of libicsum.so on one box
# (tools/bench_configs.py --only $1 per build and round; rows tagged with the build)
# usage: bash tools/probe/ab_libs.sh ROWS ROUNDS lib1.so lib2.so [...]
set -e
L=tcpip_network_protocol_stack_amd/libicsum.so
cp $L /tmp/libicsum_keep.so
trap 'cp /tmp/libicsum_keep.so $L' EXIT  # the in-tree build back whatever happens
rows=$1; rounds=$2; shift 2
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    cp $v $L
    timeout -k 10 200 python tools/bench_configs.py --only $rows | sed "s|^{|{\"lib\": \"$(basename $v)\", |"
  done
done
