set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_next.py > gpurun_out/t12.log 2>&1 &&
timeout -k 10 420 python -u bench.py --no-cpu-baseline --no-pipeline > gpurun_out/b12.json 2> gpurun_out/b12.err && echo done12
