# In-kernel clock splits of k_fast_cell / k_orient_desc (ORB_TIMING variant) on warm batches.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ORB_SLAM2_AMD_LIB=$GRAFT_REPO_ROOT/orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so timeout -k 10 120 python -u tools/ext_warm.py > gpurun_out/ext_timing.log 2>&1
tail -20 gpurun_out/ext_timing.log
