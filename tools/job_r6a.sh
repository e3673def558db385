set -o pipefail
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 200 --timeout-method thread -k "gemm_bf16 or attention" > gpurun_out/r6a_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r6a_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6a_model.log 2>&1; rc=$?; tail -8 gpurun_out/r6a_model.log
for L in vit.rs_amd/build_attnold/libvit_hip.so vit.rs_amd/libvit_hip.so vit.rs_amd/build_attnold/libvit_hip.so vit.rs_amd/libvit_hip.so; do echo "== $L"; VIT_LIB=$L timeout -k 10 120 python3 tools/bench_attn.py --colsum 2>&1 | tail -3 || exit 1; done > gpurun_out/r6a_attn.log 2>&1
timeout -k 10 400 python3 tools/ab_step.py "gemm_variant=7|gemm_variant=11" --rounds 5 --steps 4 > gpurun_out/r6a_ab.log 2>&1; tail -4 gpurun_out/r6a_ab.log
