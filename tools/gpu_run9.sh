set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_model.py -k "fused_epilogues or bf16 or smoke or reduces_loss or full_size" > gpurun_out/t9.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_gemm.py --variants 2 --modes 0,2 --rounds 3 --only fwd_qkv,fwd_proj,fwd_fc,fwd_fcproj,dgrad_fcproj,dgrad_fc > gpurun_out/bg9.log 2>&1 &&
timeout -k 10 420 python -u bench.py --no-cpu-baseline > gpurun_out/b9.json 2> gpurun_out/b9.err && echo done9
