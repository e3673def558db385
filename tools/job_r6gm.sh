# round 6: grouped tile order (VIT_GEMM_GM: unset = 8 for K <= 768, else forced for every GEMM) in the train step
set -o pipefail
for r in 1 2; do
  for g in def 4 16; do
    if [ $g = def ]; then unset VIT_GEMM_GM; else export VIT_GEMM_GM=$g; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timing > gpurun_out/r6gm_${r}_$g.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('b16 gm', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r6gm_${r}_$g.json $g
  done
done
