# round 6: weight-gradient split-K sized for fewer slots (VIT_G4_SLOTS): fewer slab bytes, the wgrad stream on part of the GPU
set -o pipefail
for r in 1 2 3; do
  for sl in 384 320 448; do
    VIT_G4_SLOTS=$sl timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timing > gpurun_out/r6s_b16_${r}_$sl.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('b16 g4 slots', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6s_b16_${r}_$sl.json $sl
  done
done
