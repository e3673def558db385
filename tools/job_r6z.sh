# round 6: persistent GEMM grid (VIT_PERSIST_CUS) 256 vs 240 vs 224, ViT-B/16 bf16 and ViT-H/14 fp8
set -o pipefail
for r in 1 2; do
  for c in 256 240 224; do
    VIT_PERSIST_CUS=$c timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timing > gpurun_out/r6z_b16_${r}_$c.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('b16 persist', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6z_b16_${r}_$c.json $c
    VIT_PERSIST_CUS=$c timeout -k 10 300 python3 bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 6 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/r6z_h14_${r}_$c.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('h14 fp8 persist', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6z_h14_${r}_$c.json $c
  done
done
