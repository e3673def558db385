# round 6: bf16 weight-gradient fill target 80 vs 45 (ViT-B/16, ViT-H/14 bf16)
set -o pipefail
for r in 1 2; do
  for f in 80 45; do
    VIT_G4_FILL=$f timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timing > gpurun_out/r6g4f_b16_${r}_$f.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('b16 g4 fill', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6g4f_b16_${r}_$f.json $f
    VIT_G4_FILL=$f timeout -k 10 300 python3 bench.py --model vit_h14 --batch 128 --steps 4 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/r6g4f_h14_${r}_$f.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('h14 bf16 g4 fill', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6g4f_h14_${r}_$f.json $f
  done
done
