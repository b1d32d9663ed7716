set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pose_gpu.py -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/t_pose.log 2>&1
bash tools/gpu_prof2.sh
echo ok
