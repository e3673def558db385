set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --model vit_h14 --batch 128 --steps 3 --warmup 1 --no-cpu-baseline --no-pipeline > gpurun_out/b20_h14.json 2> gpurun_out/b20_h14.err && echo bench20 ok
