#!/bin/bash
# Round profile on the GPU box:  bash tools/profile.sh r01
#   1. bench.py (default run, with cpu_baseline)                 -> gpurun_out/<tag>/bench.json
#   2. rocprofv3 --kernel-trace --stats over a short bench.py --serial run (kernels one at a
#      time, as in bench.py's per-kernel roofline pass)        -> gpurun_out/<tag>/ktrace/
#   3. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic per dispatch
# Every GPU step has its own time limit and the steps are chained with &&: the first failure
# ends the script.  Summarise afterwards (on any host) with tools/summarize_profile.py <tag>.
set -u
TAG=${1:-r01}
STEPS=${STEPS:-5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 420 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo "bench ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ktrace" -o run --output-format csv \
    -- python3 bench.py --serial --steps "$STEPS" --warmup 2 --no-cpu-baseline --no-pipeline > "$OUT/ktrace_bench.json" 2> "$OUT/ktrace.err" &&
echo "ktrace ok" &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv \
    -- python3 bench.py --serial --steps 1 --warmup 1 --no-cpu-baseline --no-timing --no-pipeline > /dev/null 2> "$OUT/pmc_fetch.err" &&
echo "pmc fetch ok" &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv \
    -- python3 bench.py --serial --steps 1 --warmup 1 --no-cpu-baseline --no-timing --no-pipeline > /dev/null 2> "$OUT/pmc_write.err" &&
echo "pmc write ok"
