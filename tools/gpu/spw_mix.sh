set -euo pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/spw2
for v in 16 8208 4112; do
  ICSUM_TWOCLASS=$v AB_LANE1=1 timeout -k 10 200 python3 -u tools/ab_ipv4_mix.py 0.875,0.75,0.625,0.5,0.4375 > gpurun_out/spw2/mix_$v.jsonl 2> gpurun_out/spw2/mix_$v.err
done
