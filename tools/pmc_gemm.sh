#!/bin/bash
# PMC passes over tools/bench_gemm.py (one counter group per rocprofv3 run): per-dispatch LDS,
# wait and MFMA counters of the GEMM engine -> gpurun_out/pmc_gemm/p<i>/. Args go to bench_gemm.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_gemm
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
i=0
for p in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --kernel-trace -d "$OUT/p$i" -o run --output-format csv \
      -- python3 tools/bench_gemm.py --iters 2 --rounds 1 --variants 2 "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
