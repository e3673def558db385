# early per-chunk SGD inside train_step: GPU tests, same-process A/B (bf16 B/16, fp8 H/14)
set -o pipefail
bash tools/gpu_job.sh tests || exit 1
timeout -k 10 600 python3 tools/ab_step.py "early_sgd=1|early_sgd=0" --rounds 5 --steps 4 > gpurun_out/r6esgd_ab.txt 2>&1 || exit 1
cat gpurun_out/r6esgd_ab.txt
timeout -k 10 600 python3 tools/ab_step.py "early_sgd=1|early_sgd=0" --rounds 2 --steps 2 --model vit_h14 --batch 128 --dtype fp8 > gpurun_out/r6esgd_ab_fp8.txt 2>&1 || exit 1
cat gpurun_out/r6esgd_ab_fp8.txt
