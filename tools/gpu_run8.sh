set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_gemm.py --variants 2,4 --modes 0,2 --rounds 3 > gpurun_out/bg8.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_step.py "microbatch=2|microbatch=1|concurrency=0" --rounds 4 --steps 3 > gpurun_out/ab8.log 2>&1 && echo done8
