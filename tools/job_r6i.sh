# round 6: fused residual-gradient LayerNorm backward -> MX (fp8): byte identity, gates, in-step A/B
set -o pipefail
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fp8.py -m gpu -q --timeout 120 --timeout-method thread -k "layernorm_backward_mx or layernorm_forward_mx" > gpurun_out/r6i_unit.log 2>&1; rc=$?; tail -3 gpurun_out/r6i_unit.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_model.py tests/test_gpu_production.py tests/test_gpu_fullsize.py tests/test_gpu_benchshape.py -m gpu -q --timeout 300 --timeout-method thread -k "fp8 or mx or FP8 or h14" > gpurun_out/r6i_gates.log 2>&1; rc=$?; tail -5 gpurun_out/r6i_gates.log
timeout -k 10 500 python3 tools/ab_step.py "fp8_lnb_mx=1|fp8_lnb_mx=0" --model vit_h14 --batch 128 --dtype fp8 --rounds 4 --steps 3 > gpurun_out/r6i_ab.log 2>&1; tail -3 gpurun_out/r6i_ab.log
exit $rc
