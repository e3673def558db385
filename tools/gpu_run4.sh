set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench4.json 2> gpurun_out/bench4.err
