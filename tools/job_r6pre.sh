# side pre-work (gradient clear + transposed weights on s2 beside the forward): GPU tests, same-process A/B
set -o pipefail
bash tools/gpu_job.sh tests || exit 1
timeout -k 10 600 python3 tools/ab_step.py "pre_side=1|pre_side=0" --rounds 5 --steps 4 > gpurun_out/r6pre_ab.txt 2>&1 || exit 1
cat gpurun_out/r6pre_ab.txt
timeout -k 10 600 python3 tools/ab_step.py "pre_side=1|pre_side=0" --rounds 3 --steps 2 --model vit_h14 --batch 128 --dtype fp8 > gpurun_out/r6pre_ab_fp8.txt 2>&1 || exit 1
cat gpurun_out/r6pre_ab_fp8.txt
