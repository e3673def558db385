# round 6: VIT_G4_SLOTS 512 vs 448 on ViT-L/16 and ViT-H/14 bf16 (the other configs on the g4 weight-gradient engine)
set -o pipefail
for r in 1 2; do
  for sl in 512 448; do
    VIT_G4_SLOTS=$sl timeout -k 10 300 python3 bench.py --model vit_l16 --batch 256 --steps 6 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/r6t_l16_${r}_$sl.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('l16 g4 slots', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6t_l16_${r}_$sl.json $sl
    VIT_G4_SLOTS=$sl timeout -k 10 300 python3 bench.py --model vit_h14 --batch 128 --steps 4 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/r6t_h14_${r}_$sl.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('h14 bf16 g4 slots', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6t_h14_${r}_$sl.json $sl
  done
done
