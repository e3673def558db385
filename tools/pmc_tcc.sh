#!/bin/bash
# L2 / fabric request counters of the GEMM engine (where a kernel's reads beyond
# its algorithmic bytes come from).  One counter group per rocprofv3 run over tools/bench_gemm.py;
# args go to bench_gemm.py -> gpurun_out/pmc_tcc/p<i>/.
#   p1  TCC_HIT / TCC_MISS                 L2 hit rate
#   p2  TCC_EA0_RDREQ / TCC_EA0_RDREQ_DRAM  fabric read requests, and those that reach DRAM (the
#                                          difference is served by the Infinity Cache)
#   p3  TCC_EA0_WRREQ / TCC_EA0_WRREQ_64B  fabric write requests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_tcc
mkdir -p "$OUT"
i=0
for p in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --kernel-trace -d "$OUT/p$i" -o run --output-format csv \
      -- python3 tools/bench_gemm.py --iters 2 --rounds 1 --variants 2 "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
