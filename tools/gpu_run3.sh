set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/gpmc1 -o run -- python3 tools/bench_gemm.py --no-epi --variants 2 --rounds 1 --iters 2 --only fwd_qkv,dgrad_fc,wgrad_fc > gpurun_out/gpmc1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-trace -d gpurun_out/gpmc2 -o run -- python3 tools/bench_gemm.py --no-epi --variants 2 --rounds 1 --iters 2 --only fwd_qkv,dgrad_fc,wgrad_fc > gpurun_out/gpmc2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/gpmc3 -o run -- python3 tools/bench_gemm.py --no-epi --variants 2 --rounds 1 --iters 2 --only fwd_qkv,dgrad_fc,wgrad_fc > gpurun_out/gpmc3.log 2>&1
