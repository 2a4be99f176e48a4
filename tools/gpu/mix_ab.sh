set -e
L=tcpip_network_protocol_stack_amd/libicsum.so
cp $L /tmp/libicsum_keep.so
for V in build_ab/libicsum_prev.so /tmp/libicsum_keep.so; do
  cp $V $L
  timeout -k 10 120 python3 tools/ab_mix_split.py 1048576 0.1875,0.25,0.5,0.625,0.6875,0.75,0.875 | sed "s|^{|{\"lib\": \"$(basename $V)\", \"forced\": 0, |"
  ICSUM_FORCE=twoclass=16 timeout -k 10 120 python3 tools/ab_mix_split.py 1048576 0.125 | sed "s|^{|{\"lib\": \"$(basename $V)\", \"forced\": 1, |"
done
cp /tmp/libicsum_keep.so $L
