set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_gemm.py --variants 2 --modes 0,512,768,1280,1536 --rounds 3 --only fwd_proj,fwd_fc,fwd_fcproj,dgrad_fcproj > gpurun_out/bg10.log 2>&1 && echo done10
