# round 6: LayerNorm forward -> MX with whole rounds of tiles + leftover rows: identity, gates, timing
set -o pipefail
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fp8.py -m gpu -q --timeout 120 --timeout-method thread -k "layernorm_backward_mx or layernorm_forward_mx" > gpurun_out/r6l_unit.log 2>&1; rc=$?; tail -3 gpurun_out/r6l_unit.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/bench_lnmx.py --rows 16384,16448,32896 || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_model.py tests/test_gpu_production.py tests/test_gpu_benchshape.py -m gpu -q --timeout 300 --timeout-method thread -k "fp8 or FP8 or h14" > gpurun_out/r6l_gates.log 2>&1; rc=$?; tail -3 gpurun_out/r6l_gates.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --model vit_h14 --batch 128 --dtype fp8 --no-cpu-baseline > gpurun_out/r6l_h14_fp8.json 2> gpurun_out/r6l_h14_fp8.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r6l_h14_fp8.json')); k=d['kernels']; print(d['value'], d['ms_per_step'], 'quant', k['quantize_mx']['ms_per_step'], 'lnb', k['layernorm_bwd']['ms_per_step'], 'lnf', k['layernorm_fwd']['ms_per_step'])"
