#!/bin/bash
# Round 3: every dev A/B tool converted to ICSUM_FORCE runs once at reduced
# rounds (each variant's outputs are compared inside the tool), so a stale or
# mistyped force key shows up as an ics_create failure here.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3_tools}; mkdir -p $O
run() {  # tag, then the command
  tag=$1; shift
  echo "== $tag"
  timeout -k 10 240 "$@" > $O/$tag.jsonl 2> $O/$tag.err
}
run ab_tiny python3 -u tools/ab_tiny.py
run ab_bins python3 -u tools/ab_bins.py --rounds 1 --iters 3
run ab_lastbin python3 -u tools/ab_lastbin.py --var bin --caps=-1,1 --workloads config4,ack --rounds 1 --iters 3
run ab_lastbin_plan python3 -u tools/ab_lastbin.py --var bin_plan --caps=-1,0,1,2,3 --workloads bimodal --rounds 1 --iters 3
run ab_small_offsets python3 -u tools/ab_small_offsets.py
run ab_ipv4_offsets python3 -u tools/ab_ipv4_offsets.py --rounds 1 --iters 5
run ab_ipv4_geom python3 -u tools/ab_ipv4_geom.py 16x8x3,32x4x3
run ab_ipv4_mix python3 -u tools/ab_ipv4_mix.py 0.5
run ab_wrap_ack python3 -u tools/ab_wrap_ack.py
run ab_wrap_twopass python3 -u tools/ab_wrap_twopass.py
run ab_xcd python3 -u tools/ab_xcd.py --workloads ns --rounds 2 --iters 5
run sweep_geometry python3 -u tools/sweep_geometry.py --workloads ns,tcp64 --rounds 1 --iters 3
run ab_host python3 -u tools/ab_host.py --variants 2x64,3x32 --rounds 1
echo "all tools ran"
