# round 6: weight-gradient split rule (VIT_G4_RULE 1 = one round >= 80 %, 0 = round-5 rule) on B/16, L/16, H/14 bf16
set -o pipefail
for r in 1 2; do
  for ru in 1 0; do
    VIT_G4_RULE=$ru timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timing > gpurun_out/r6u_b16_${r}_$ru.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('b16 g4 rule', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6u_b16_${r}_$ru.json $ru
    VIT_G4_RULE=$ru timeout -k 10 300 python3 bench.py --model vit_l16 --batch 256 --steps 6 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/r6u_l16_${r}_$ru.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('l16 g4 rule', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6u_l16_${r}_$ru.json $ru
    VIT_G4_RULE=$ru timeout -k 10 300 python3 bench.py --model vit_h14 --batch 128 --steps 4 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/r6u_h14_${r}_$ru.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('h14 bf16 g4 rule', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6u_h14_${r}_$ru.json $ru
  done
done
