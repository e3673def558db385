#!/bin/bash
# One parameterised runner for the GPU box (replaces the per-experiment gpu_run*.sh scripts).
#   gpurun -- bash tools/gpu_job.sh <job> [args...]
# jobs (every GPU step has its own time limit; steps chain with &&, so the first failure ends it):
#   tests [pytest args]   python -m pytest -m gpu (default: all GPU tests) -> gpurun_out/tests.<stamp>.log
#   smoke                 __graft_entry__.smoke()                          -> gpurun_out/smoke.<stamp>.log
#   bench [bench args]    python bench.py ...                              -> gpurun_out/bench.<stamp>.json
# Every call writes its own timestamped log (<stamp> = UTC date-time + pid), so a run that is
# killed leaves its log next to the retry's (gpurun_out/ is merged back, never overwritten); the
# un-stamped names are symlinks to the newest one.
#   attn [bench_attn args] tools/bench_attn.py                             -> stdout
#   gemm [bench_gemm args] tools/bench_gemm.py                             -> stdout
#   profile TAG           tools/profile.sh TAG (bench + rocprofv3 stats + PMC passes)
#   ktrace TAG [bench args]  rocprofv3 --kernel-trace --stats of one bench.py run -> gpurun_out/TAG/
#   py SCRIPT [args]      python3 SCRIPT args (any tool under tools/)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
job=${1:?job}; shift
stamp=$(date -u +%Y%m%dT%H%M%S).$$
keep() { ln -sfn "$(basename "$1")" "gpurun_out/$2"; }
case "$job" in
  tests)
    log=gpurun_out/tests.$stamp.log; keep "$log" tests.log
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
        > "$log" 2>&1; rc=$?; tail -25 "$log"; exit $rc ;;
  smoke)
    log=gpurun_out/smoke.$stamp.log; keep "$log" smoke.log
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee "$log" ;;
  bench)
    out=gpurun_out/bench.$stamp.json; keep "$out" bench.json; keep "gpurun_out/bench.$stamp.err" bench.err
    timeout -k 10 600 python3 bench.py "$@" > "$out" 2> "gpurun_out/bench.$stamp.err"; rc=$?
    cat "$out"; tail -5 "gpurun_out/bench.$stamp.err"; exit $rc ;;
  attn)
    timeout -k 10 300 python3 tools/bench_attn.py "$@" 2>&1 | tee "gpurun_out/attn.$stamp.log" ;;
  gemm)
    timeout -k 10 300 python3 tools/bench_gemm.py "$@" 2>&1 | tee "gpurun_out/gemm.$stamp.log" ;;
  profile)
    bash tools/profile.sh "$@" ;;
  ktrace)
    tag=${1:?tag}; shift
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "gpurun_out/$tag" -o run --output-format csv \
        -- python3 bench.py "$@" > "gpurun_out/$tag.json" 2> "gpurun_out/$tag.err" && echo "ktrace $tag ok" ;;
  py)
    script=${1:?script}; shift
    timeout -k 10 600 python3 "$script" "$@" 2>&1 | tee "gpurun_out/py.$(basename "$script" .py).$stamp.log" ;;
  *) echo "unknown job $job"; exit 2 ;;
esac
