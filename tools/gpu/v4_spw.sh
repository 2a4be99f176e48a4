#!/bin/bash
# Fused two-class IPv4 launch at 64 / 32 / 16 datagrams per wave, forced, over the ACK-share sweep.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/v4spw; mkdir -p $O
for w in 64 32 16; do
  ICSUM_TWOCLASS=16 ICSUM_V4_SPW=$w AB_LANE1=1 timeout -k 10 200 python3 -u tools/ab_ipv4_mix.py 0.75,0.5,0.4375,0.3125,0.25 > $O/mix_$w.jsonl 2> $O/mix_$w.err
done
