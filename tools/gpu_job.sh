#!/bin/bash
# One parameterised runner for the GPU box (replaces the per-experiment gpu_run*.sh scripts).
#   gpurun -- bash tools/gpu_job.sh <job> [args...]
# jobs (every GPU step has its own time limit; steps chain with &&, so the first failure ends it):
#   tests [pytest args]   python -m pytest -m gpu (default: all GPU tests) -> gpurun_out/tests.log
#   smoke                 __graft_entry__.smoke()                          -> gpurun_out/smoke.log
#   bench [bench args]    python bench.py ...                              -> gpurun_out/bench.json
#   attn [bench_attn args] tools/bench_attn.py                             -> stdout
#   gemm [bench_gemm args] tools/bench_gemm.py                             -> stdout
#   profile TAG           tools/profile.sh TAG (bench + rocprofv3 stats + PMC passes)
#   ktrace TAG [bench args]  rocprofv3 --kernel-trace --stats of one bench.py run -> gpurun_out/TAG/
#   py SCRIPT [args]      python3 SCRIPT args (any tool under tools/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
job=${1:?job}; shift
case "$job" in
  tests)
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
        > gpurun_out/tests.log 2>&1; rc=$?; tail -25 gpurun_out/tests.log; exit $rc ;;
  smoke)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/smoke.log ;;
  bench)
    timeout -k 10 600 python3 bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
    cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err; exit $rc ;;
  attn)
    timeout -k 10 300 python3 tools/bench_attn.py "$@" ;;
  gemm)
    timeout -k 10 300 python3 tools/bench_gemm.py "$@" ;;
  profile)
    bash tools/profile.sh "$@" ;;
  ktrace)
    tag=${1:?tag}; shift
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "gpurun_out/$tag" -o run --output-format csv \
        -- python3 bench.py "$@" > "gpurun_out/$tag.json" 2> "gpurun_out/$tag.err" && echo "ktrace $tag ok" ;;
  py)
    script=${1:?script}; shift
    timeout -k 10 600 python3 "$script" "$@" ;;
  *) echo "unknown job $job"; exit 2 ;;
esac
