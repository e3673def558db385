# round 6: HIP hardware queues per process (GPU_MAX_HW_QUEUES, default 4) vs 8 with the trainer's 4-5 streams
set -o pipefail
for r in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timing > gpurun_out/r6y_b16_${r}_$q.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('b16 hwq', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6y_b16_${r}_$q.json $q
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 6 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/r6y_h14_${r}_$q.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('h14 fp8 hwq', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6y_h14_${r}_$q.json $q
  done
done
timeout -k 10 500 python3 tools/ab_step.py "microbatch=2|microbatch=1" --rounds 4 --steps 4 2>&1 | tail -2
