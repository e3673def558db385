set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t16.log 2>&1 &&
echo tests16 ok &&
timeout -k 10 420 python -u bench.py > gpurun_out/b16.json 2> gpurun_out/b16.err && echo bench16 ok &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke16.log 2>&1 && echo smoke16 ok
