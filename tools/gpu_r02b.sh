# octree / fast_cell phase stamps (ORB_TIMING variant) + single-stream kernel stats
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ORB_SLAM2_AMD_LIB=orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so timeout -k 10 120 python -u tools/fast_timing.py > gpurun_out/timing.log 2>&1
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_1s -o bench -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 20 --warmup 5 --no-lba --no-extras --no-stereo --streams 1 --batch 64 > $GRAFT_REPO_ROOT/gpurun_out/prof_1s.log 2>&1
echo r02b ok
