set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_step.py "gemm_debug=0|gemm_debug=8|gemm_debug=16" --rounds 4 --steps 3 > gpurun_out/ab3.log 2>&1
