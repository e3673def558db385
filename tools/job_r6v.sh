# round 6: gates for the bf16 weight-gradient split rule, then the fp8 split-rule A/B (ViT-H/14 fp8)
set -o pipefail
bash tools/gpu_job.sh tests > /dev/null 2>&1; rc=$?; tail -2 gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for ru in 1 0; do
    VIT_F8_SPLIT_RULE=$ru timeout -k 10 300 python3 bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 6 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/r6v_h14_${r}_$ru.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('h14 fp8 split rule', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6v_h14_${r}_$ru.json $ru
  done
done
