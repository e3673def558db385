# round 6: fp8 streaming engine with one phase per K-step as the default: gates + in-step A/B (ViT-H/14 fp8)
set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_model.py tests/test_gpu_production.py tests/test_gpu_benchshape.py -m gpu -q --timeout 300 --timeout-method thread -k "fp8 or mx or FP8 or h14" > gpurun_out/r6g_gates.log 2>&1; rc=$?; tail -3 gpurun_out/r6g_gates.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for L in vit.rs_amd/libvit_hip.so vit.rs_amd/build_f8two/libvit_hip.so; do
    n=$(basename $(dirname $L))
    VIT_LIB=$L timeout -k 10 300 python3 bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r6g_h14_${r}_$n.json 2> gpurun_out/r6g_h14_${r}_$n.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print(sys.argv[2], d['value'], d['ms_per_step'], {n: k[n]['ms_per_step'] for n in ('gemm_fc_fwd','gemm_qkv_fwd','gemm_fc_dgrad','gemm_fcproj_fwd','gemm_fcproj_dgrad','gemm_qkv_dgrad')})" gpurun_out/r6g_h14_${r}_$n.json $n
  done
done
VIT_LIB=vit.rs_amd/build_f8trace/libvit_hip.so timeout -k 10 200 python3 tools/f8_trace.py --only fwd_qkv,dgrad_fc,fwd_fc,fwd_proj,dgrad_qkv,fwd_fcproj > gpurun_out/r6g_f8trace.log 2>&1 || exit 1
