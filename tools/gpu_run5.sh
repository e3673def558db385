set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "fused_epilogues or layouts or matmul_bf16" > gpurun_out/t5.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_gemm.py --variants 2 --modes 0,32 --rounds 3 > gpurun_out/bg5.log 2>&1 &&
timeout -k 10 400 python -u tools/ab_step.py "gemm_debug=0|gemm_debug=32" --rounds 4 --steps 3 > gpurun_out/ab5.log 2>&1
