# round 6 final (final code: head path, patch tail, side pre-work): GPU tests, smoke, profile r06g (bench + rocprofv3 stats + traffic), other configs
set -o pipefail
bash tools/gpu_job.sh tests || exit 1
bash tools/gpu_job.sh smoke || exit 1
bash tools/profile.sh r06g || exit 1
for cfg in "vit_h14 128 fp8" "vit_h14 128 bf16" "vit_l16 256 bf16"; do
  set -- $cfg
  timeout -k 10 400 python3 bench.py --model $1 --batch $2 --dtype $3 --no-cpu-baseline > gpurun_out/r06g_${1}_$3.json 2> gpurun_out/r06g_${1}_$3.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/r06g_${1}_$3.json
done
