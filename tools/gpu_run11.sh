set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_model.py -k "layernorm or bf16 or reduces_loss or full_size or golden or oracle" > gpurun_out/t11.log 2>&1 &&
timeout -k 10 420 python -u bench.py --no-cpu-baseline --no-pipeline > gpurun_out/b11.json 2> gpurun_out/b11.err && echo done11
