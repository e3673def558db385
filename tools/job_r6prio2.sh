# round 6: stream priorities re-checked after the 45 % one-round weight-gradient splits
set -o pipefail
for r in 1 2; do
  for p in 2 0; do
    VIT_STREAM_PRIO=$p timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timing > gpurun_out/r6pr_b16_${r}_$p.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('b16 prio', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6pr_b16_${r}_$p.json $p
  done
  for p in 0 2; do
    VIT_STREAM_PRIO=$p timeout -k 10 300 python3 bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 6 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/r6pr_h14_${r}_$p.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('h14 fp8 prio', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6pr_h14_${r}_$p.json $p
  done
done
