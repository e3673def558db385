set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_step.py "microbatch=2|microbatch=1|microbatch=4|microbatch=2,gemm_variant=4" --rounds 4 --steps 3 > gpurun_out/ab17.log 2>&1 && echo ab17 ok
