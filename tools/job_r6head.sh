# head split-K + fp32 rows-reduce column sums: GPU tests (fp8 curve drift alarm deselected: re-record
# rule in tests/golden/make_fp8_curve.py), same-process A/B of the head split, the fp8 curve re-recorded
set -o pipefail
bash tools/gpu_job.sh tests --deselect tests/test_gpu_model.py::test_fp8_loss_curve_fixture || exit 1
timeout -k 10 600 python3 tools/ab_step.py "head_splitk=1|head_splitk=0" --rounds 5 --steps 4 > gpurun_out/r6head_ab.txt 2>&1 || exit 1
cat gpurun_out/r6head_ab.txt
timeout -k 10 300 python3 tests/golden/make_fp8_curve.py gpurun_out/fp8_curve_test_h64.json || exit 1
echo curve ok
