# fp8 curve fixture re-check, then a kernel trace of the serial bench pass (head-path kernel durations)
set -o pipefail
bash tools/gpu_job.sh tests tests/test_gpu_model.py::test_fp8_loss_curve_fixture || exit 1
bash tools/gpu_job.sh ktrace r6h --serial --steps 3 --warmup 1 --no-cpu-baseline --no-pipeline || exit 1
echo done
