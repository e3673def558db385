set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py -k "vit_l16 or vit_h14" > gpurun_out/t14.log 2>&1 &&
echo tests14 ok &&
timeout -k 10 400 python -u bench.py --model vit_l16 --no-cpu-baseline --no-pipeline > gpurun_out/b14_l16.json 2> gpurun_out/b14_l16.err && echo bench14 ok
