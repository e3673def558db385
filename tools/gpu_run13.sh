set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t13.log 2>&1 &&
echo tests13 ok &&
bash tools/profile.sh r01e
