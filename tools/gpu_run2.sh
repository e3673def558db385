set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_wt.log 2>&1
