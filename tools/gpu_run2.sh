set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/loss_traj.py 0.5 > gpurun_out/traj.log 2>&1 &&
VIT_LIB=$PWD/tools/_old/libvit_hip.so timeout -k 10 120 python -u tools/loss_traj.py 0.5 >> gpurun_out/traj.log 2>&1 &&
timeout -k 10 120 python -u tools/loss_traj.py 0.2 >> gpurun_out/traj.log 2>&1
