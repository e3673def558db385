set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/h14
timeout -k 10 400 python3 bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 5 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/h14/fp8.json 2> gpurun_out/h14/fp8.err &&
VIT_FP8_WGRAD=0 timeout -k 10 400 python3 bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 5 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/h14/fp8_bf16wgrad.json 2> gpurun_out/h14/fp8_bf16wgrad.err
