set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_step.py "dgrad_transposed=1|dgrad_transposed=0|microbatch=1|microbatch=2,concurrency=0|concurrency=1" --rounds 4 --steps 3 > gpurun_out/ab1.log 2>&1
