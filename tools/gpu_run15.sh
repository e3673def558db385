set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "attention or error_channel" > gpurun_out/t15a.log 2>&1 &&
echo ops15 ok &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py -k "vit_h14" > gpurun_out/t15b.log 2>&1 &&
echo model15 ok &&
timeout -k 10 400 python -u bench.py --model vit_h14 --batch 128 --steps 3 --warmup 1 --no-cpu-baseline --no-pipeline > gpurun_out/b15_h14.json 2> gpurun_out/b15_h14.err && echo bench15 ok
