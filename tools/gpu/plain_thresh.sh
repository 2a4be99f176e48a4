#!/bin/bash
# Plain checksum of raw-datagram ACK mixes below the two-class threshold: AUTO vs two-class forced (16 / 32 per wave).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/pth; mkdir -p $O
timeout -k 10 200 python3 -u tools/ab_ipv4_mix.py 0.375,0.3125,0.25,0.1875 > $O/auto.jsonl 2> $O/auto.err
for v in 4112 8208; do
  ICSUM_TWOCLASS=$v timeout -k 10 200 python3 -u tools/ab_ipv4_mix.py 0.375,0.3125,0.25,0.1875 > $O/two_$v.jsonl 2> $O/two_$v.err
done
