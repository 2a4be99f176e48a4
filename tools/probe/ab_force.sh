# dev: interleaved A/B of ICSUM_FORCE settings on one build (tools/bench_configs.py --only $1 per setting and round)
# usage: bash tools/probe/ab_force.sh ROWS ROUNDS "" "lps=16,unroll=7" [...]   ("" = the default dispatch)
set -e
rows=$1; rounds=$2; shift 2
for r in $(seq 1 $rounds); do
  for f in "$@"; do
    ICSUM_FORCE="$f" timeout -k 10 200 python tools/bench_configs.py --only $rows | sed "s|^{|{\"force\": \"$f\", |"
  done
done
