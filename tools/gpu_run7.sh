set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_gemm.py --variants 2 --modes 0,1024,1536,2048,3072 --rounds 3 --only fwd_qkv,fwd_proj,fwd_fc,fwd_fcproj,dgrad_fcproj,dgrad_fc > gpurun_out/bg7.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_step.py "gemm_debug=0|gemm_debug=1024|gemm_debug=1536|gemm_debug=2048" --rounds 4 --steps 3 > gpurun_out/ab7.log 2>&1 &&
bash tools/profile.sh r01d && echo done7
