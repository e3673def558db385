# ViT-B/16 bf16: weight-gradient split fill target 35 / 45 / 60 %, interleaved bench.py rounds on one box
set -o pipefail
for r in 1 2; do
  for f in 35 45 60; do
    VIT_G4_FILL=$f timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/g4f_${f}_$r.json 2> gpurun_out/g4f_${f}_$r.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('fill', sys.argv[2], 'round', sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/g4f_${f}_$r.json $f $r
  done
done
