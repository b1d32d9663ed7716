set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export ORB_SLAM2_AMD_LIB=$GRAFT_REPO_ROOT/orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so
timeout -k 5 120 python -u tools/lba_timing.py solves=3 > gpurun_out/lba_timing_df.log 2>&1
grep "ldlt_df" gpurun_out/lba_timing_df.log | tail -4
