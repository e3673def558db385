# round 6: fp8 weight-gradient one-round fill target (VIT_F8_FILL) 80 / 60 / 45 on ViT-H/14 fp8
set -o pipefail
for r in 1 2; do
  for f in 45 35 25; do
    VIT_F8_FILL=$f timeout -k 10 300 python3 bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 6 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/r6f8fill_${r}_$f.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('h14 fp8 fill', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6f8fill_${r}_$f.json $f
  done
done
