set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ORB_SLAM2_AMD_LIB=orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so timeout -k 10 120 python -u bench.py --no-cpu --no-lba --no-extras --no-stereo --no-profile --steps 2 --warmup 1 --streams 1 --batch 64 --no-match-stream > gpurun_out/timing_sfi.log 2>&1
echo ok
