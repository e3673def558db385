# final binary (early SGD on in fp8 mode): GPU tests, smoke, ViT-H/14 fp8 and ViT-B/16 bench
set -o pipefail
bash tools/gpu_job.sh tests || exit 1
bash tools/gpu_job.sh smoke || exit 1
timeout -k 10 400 python3 bench.py --model vit_h14 --batch 128 --dtype fp8 --no-cpu-baseline > gpurun_out/r06h_vit_h14_fp8.json 2> gpurun_out/r06h_vit_h14_fp8.err || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/r06h_vit_h14_fp8.json
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/r06h_bench.json 2> gpurun_out/r06h_bench.err || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])" gpurun_out/r06h_bench.json
