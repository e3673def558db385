set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/r01e_mfma -o run --output-format csv \
    -- python3 bench.py --serial --steps 1 --warmup 1 --no-cpu-baseline --no-timing --no-pipeline > /dev/null 2> gpurun_out/r01e_mfma.err && echo mfma ok
