set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 5 120 python -u tools/pose_timing.py 5 > gpurun_out/pose_timing_base.log 2>&1
ORB_SLAM2_AMD_LIB=$GRAFT_REPO_ROOT/orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so timeout -k 5 120 python -u tools/pose_timing.py 3 > gpurun_out/pose_timing.log 2>&1
cat gpurun_out/pose_timing_base.log gpurun_out/pose_timing.log | grep -v amdgpu.ids
