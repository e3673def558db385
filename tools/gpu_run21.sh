set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/h14_ktrace -o run --output-format csv \
    -- python3 bench.py --model vit_h14 --batch 128 --serial --steps 2 --warmup 1 --no-cpu-baseline --no-timing --no-pipeline > gpurun_out/h14_ktrace.json 2> gpurun_out/h14_ktrace.err && echo ktrace21 ok
