# early per-chunk SGD (on s_comm) A/B repeated on a second box: ViT-B/16 bf16, ViT-H/14 fp8, ViT-L/16 bf16
set -o pipefail
timeout -k 10 600 python3 tools/ab_step.py "early_sgd=1|early_sgd=0" --rounds 5 --steps 4 > gpurun_out/r6esgd2_b16.txt 2>&1 || exit 1
cat gpurun_out/r6esgd2_b16.txt
timeout -k 10 600 python3 tools/ab_step.py "early_sgd=1|early_sgd=0" --rounds 2 --steps 2 --model vit_h14 --batch 128 --dtype fp8 > gpurun_out/r6esgd2_h14.txt 2>&1 || exit 1
cat gpurun_out/r6esgd2_h14.txt
timeout -k 10 600 python3 tools/ab_step.py "early_sgd=1|early_sgd=0" --rounds 2 --steps 2 --model vit_l16 --batch 256 > gpurun_out/r6esgd2_l16.txt 2>&1 || exit 1
cat gpurun_out/r6esgd2_l16.txt
