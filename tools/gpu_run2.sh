set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 2 3 4; do
VIT_GEMM=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/bench_v$v.log 2>&1 || exit 1
done
