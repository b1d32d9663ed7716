set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ORB_SLAM2_AMD_LIB=orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so timeout -k 10 120 python -u tools/ldlt_warm.py > gpurun_out/ldlt_warm.log 2>&1
