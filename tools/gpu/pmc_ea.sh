#!/bin/bash
# Memory-side (TCC_EA0) request counters for the kernels that store into the
# datagrams: k_ipv4_tcp COMPUTE vs PATCH (config 2), k_router_ttl, k_tcp_wrap
# in place vs headers apart.  Four TCC counters per pass.  Usage: pmc_ea.sh OUTDIR
set -euo pipefail
OUT=$(realpath -m "$1"); mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
BC="tools/bench_configs.py --settle-ms 0 --rounds 1 --iters 2"
WR="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum"
RD="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
ST="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum"
run() {  # name, counters, bench_configs args
  timeout -s KILL 200 rocprofv3 --pmc $2 --output-format csv -d "$OUT/$1" -o pmc -- python3 $BC $3 \
    > "$OUT/$1.log" 2>&1
}
for g in WR RD ST; do
  run "ipv4_compute_$g" "${!g}" "--only ipv4 --modes compute"
  run "ipv4_patch_$g" "${!g}" "--only ipv4 --modes patch"
  run "router_$g" "${!g}" "--only router"
  run "wrap_$g" "${!g}" "--only wrap --wrap-device-only"
done
