set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "gemm" tests/test_gpu_model.py -k "gemm or bf16" > gpurun_out/t18.log 2>&1 &&
echo tests18 ok &&
timeout -k 10 420 python -u bench.py --no-cpu-baseline --no-pipeline > gpurun_out/b18.json 2> gpurun_out/b18.err && echo bench18 ok
