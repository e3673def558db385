set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t6.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke6.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_gemm.py --variants 2,5 --rounds 3 > gpurun_out/bg6.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_step.py "gemm_variant=2|gemm_variant=5|gemm_variant=5,concurrency=0|gemm_variant=2,concurrency=0" --rounds 4 --steps 3 > gpurun_out/ab6.log 2>&1 &&
echo done6
