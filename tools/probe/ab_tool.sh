# dev: run one measurement tool once per build of libicsum.so, rows tagged with the build
# usage: bash tools/probe/ab_tool.sh "python tools/ab_tile.py 262144" lib1.so lib2.so [...]
set -e
L=tcpip_network_protocol_stack_amd/libicsum.so
cp $L /tmp/libicsum_keep.so
cmd=$1; shift
for v in "$@"; do
  cp $v $L
  timeout -k 10 300 $cmd | sed "s|^{|{\"lib\": \"$(basename $v)\", |"
done
cp /tmp/libicsum_keep.so $L
