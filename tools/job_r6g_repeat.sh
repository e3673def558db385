# round 6 final binary (r06g code + fp8 early SGD): three default bench.py runs on one box (box-level spread of the headline)
set -o pipefail
for i in 1 2 3; do
  timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/r06g_rep$i.json 2> gpurun_out/r06g_rep$i.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('run', sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])" gpurun_out/r06g_rep$i.json $i
done
