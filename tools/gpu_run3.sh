set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/tl.log 2>&1
