# GPU session script: GEMM parity (all engines), GEMM microbench, loss trajectories, full-step bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "gemm or matmul" > gpurun_out/t1.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_gemm.py --no-epi --variants 2,3 > gpurun_out/bg.log 2>&1 &&
timeout -k 10 120 python -u tools/loss_traj.py 0.1 > gpurun_out/traj.log 2>&1 &&
timeout -k 10 120 python -u tools/loss_traj.py 0.2 >> gpurun_out/traj.log 2>&1 &&
VIT_GEMM=3 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench3.log 2>&1
