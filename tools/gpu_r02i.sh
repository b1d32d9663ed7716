set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_r02g.sh
ORB_SLAM2_AMD_LIB=orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so timeout -k 10 120 python -u tools/fast_timing.py > gpurun_out/timing.log 2>&1
echo ok
