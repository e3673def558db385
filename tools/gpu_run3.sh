set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/bench_gemm.py --no-epi --variants 2 --rounds 2 > gpurun_out/bg_norm.log 2>&1 &&
VIT_DEBUG_SAME_TILE=1 timeout -k 10 200 python3 tools/bench_gemm.py --no-epi --variants 2 --rounds 2 > gpurun_out/bg_same.log 2>&1
