# round 6: fused LayerNorm -> MX, final form: byte identity + fp8 gates, then the in-step A/B on ViT-H/14 fp8
set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_model.py tests/test_gpu_production.py tests/test_gpu_benchshape.py -m gpu -q --timeout 300 --timeout-method thread -k "fp8 or mx or FP8 or h14" > gpurun_out/r6d_gates.log 2>&1; rc=$?; tail -3 gpurun_out/r6d_gates.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 tools/ab_step.py "fp8_ln_mx=1|fp8_ln_mx=0" --model vit_h14 --batch 128 --dtype fp8 --rounds 4 --steps 3 > gpurun_out/r6d_ab.log 2>&1; tail -3 gpurun_out/r6d_ab.log
