# patch embedding backward tail (patch wgrad fill 80 %, small gradients on s2): GPU tests, same-process A/B
set -o pipefail
bash tools/gpu_job.sh tests || exit 1
timeout -k 10 600 python3 tools/ab_step.py "patch_tail=1|patch_tail=0" --rounds 5 --steps 4 > gpurun_out/r6ptail_ab.txt 2>&1 || exit 1
cat gpurun_out/r6ptail_ab.txt
