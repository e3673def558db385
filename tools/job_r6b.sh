# round 6: the oracle-anchored fp8 / attention gates on the current build, then the fp8 curve re-record
set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_model.py tests/test_gpu_fp8.py tests/test_gpu_production.py tests/test_gpu_fullsize.py tests/test_gpu_benchshape.py -m gpu -q --timeout 300 --timeout-method thread -k "not loss_curve_fixture" > gpurun_out/r6b_gates.log 2>&1; rc=$?; tail -4 gpurun_out/r6b_gates.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tests/golden/make_fp8_curve.py gpurun_out/fp8_curve_test_h64.json "r06: attention forward pairwise row sum + v_rcp / v_log (VERDICT r05 item 6)" 2>&1 | tail -2
timeout -k 10 400 python3 tools/ab_step.py "gemm_variant=7|gemm_variant=11|gemm_variant=7,microbatch=1|gemm_variant=11,microbatch=1" --rounds 4 --steps 4 > gpurun_out/r6b_ab.log 2>&1; tail -5 gpurun_out/r6b_ab.log
