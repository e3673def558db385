# round 6: gates after the LayerNorm-backward MX fusion, then the ViT-H/14 fp8 bench
set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_model.py tests/test_gpu_production.py tests/test_gpu_ops.py -m gpu -q --timeout 300 --timeout-method thread -k "config5 or fp8_loss_curve or layernorm or production" > gpurun_out/r6j_gates.log 2>&1; rc=$?; tail -4 gpurun_out/r6j_gates.log
timeout -k 10 400 python3 bench.py --model vit_h14 --batch 128 --dtype fp8 --no-cpu-baseline > gpurun_out/r6j_h14_fp8.json 2> gpurun_out/r6j_h14_fp8.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r6j_h14_fp8.json')); k=d['kernels']; print(d['value'], d['ms_per_step'], 'quant', k['quantize_mx']['ms_per_step'], 'lnb', k['layernorm_bwd']['ms_per_step'], 'lnf', k['layernorm_fwd']['ms_per_step'])"
exit $rc
