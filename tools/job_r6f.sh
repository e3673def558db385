# round 6: one phase per K-step (two barriers instead of four) in the bf16 (variant 7) and fp8 streaming engines
set -o pipefail
for r in 1 2; do
  for L in vit.rs_amd/libvit_hip.so vit.rs_amd/build_g2one/libvit_hip.so; do
    echo "== $L"; VIT_LIB=$L timeout -k 10 200 python3 tools/bench_gemm.py --variants 7 --rounds 1 || exit 1
  done
done > gpurun_out/r6f_gemm.log 2>&1
for r in 1 2; do
  for L in vit.rs_amd/libvit_hip.so vit.rs_amd/build_g2one/libvit_hip.so; do
    VIT_LIB=$L timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6f_b16_${r}_$(basename $(dirname $L)).json || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6f_b16_${r}_$(basename $(dirname $L)).json $L
  done
done >> gpurun_out/r6f_gemm.log 2>&1
tail -12 gpurun_out/r6f_gemm.log
