# dev: interleaved A/B of two builds of libicsum.so on one box (tools/bench_configs.py --only $1)
# usage: bash tools/probe/ab_lib.sh ipv4 tools/probe/libicsum_base.so tools/probe/libicsum_shfl.so [rounds]
set -e
L=tcpip_network_protocol_stack_amd/libicsum.so
cp $L /tmp/libicsum_keep.so
for r in $(seq 1 ${4:-3}); do
  for v in $2 $3; do
    cp $v $L
    timeout -k 10 200 python tools/bench_configs.py --only $1 | sed "s|^{|{\"lib\": \"$(basename $v)\", |"
  done
done
cp /tmp/libicsum_keep.so $L
