# round 6: more stream-priority modes (3: mb0 high, mb1 low, wgrad high; 4: mb0 high, mb1 low, wgrad low)
set -o pipefail
for r in 1 2; do
  for p in 2 3 4; do
    VIT_STREAM_PRIO=$p timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timing > gpurun_out/r6q_b16_${r}_$p.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('b16 prio', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6q_b16_${r}_$p.json $p
  done
done
for r in 1 2; do
  for p in 0 3 4; do
    VIT_STREAM_PRIO=$p timeout -k 10 300 python3 bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 6 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/r6q_h14_${r}_$p.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('h14 fp8 prio', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6q_h14_${r}_$p.json $p
  done
done
