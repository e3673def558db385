# round 6: fused LayerNorm -> MX (fp8): byte-identity + oracle gates, then ViT-H/14 fp8 A/B (VIT_FP8_LN_MX)
set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_model.py tests/test_gpu_production.py tests/test_gpu_benchshape.py -m gpu -q --timeout 300 --timeout-method thread -k "fp8 or mx or FP8 or h14" > gpurun_out/r6c_gates.log 2>&1; rc=$?; tail -4 gpurun_out/r6c_gates.log; [ $rc -eq 0 ] || exit $rc
VIT_FP8_LN_MX=0 timeout -k 10 400 python3 bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r6c_h14_fp8_lnmx0.json 2> gpurun_out/r6c_h14_fp8_lnmx0.err && \
timeout -k 10 400 python3 bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r6c_h14_fp8.json 2> gpurun_out/r6c_h14_fp8.err && \
python3 - <<'PY'
import json
for t in ("r6c_h14_fp8_lnmx0", "r6c_h14_fp8"):
    d = json.load(open(f"gpurun_out/{t}.json"))
    k = d["kernels"]
    print(t, d["value"], d["ms_per_step"], "quant", k["quantize_mx"]["ms_per_step"], "lnf", k["layernorm_fwd"]["ms_per_step"])
PY
