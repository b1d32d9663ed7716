# LBA parity tests, LDLT clock split (timing variant), same-box A/B against the base variant,
# and rocprofv3 kernel stats of the working tree's solve.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lba_gpu.py tests/test_global_ba.py tests/test_cpp_shim.py tests/test_lba_dist_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_lba.log 2>&1
ORB_SLAM2_AMD_LIB=orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so timeout -k 10 120 python -u tools/lba_timing.py > gpurun_out/lba_timing.log 2>&1
timeout -k 10 600 bash tools/gpu_ab_lba.sh
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_lba -o lba -- python3 $GRAFT_REPO_ROOT/tools/lba_timing.py > $GRAFT_REPO_ROOT/gpurun_out/prof_lba.log 2>&1
cd $GRAFT_REPO_ROOT && ORB_SLAM2_AMD_LIB=orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so timeout -k 10 120 python -u tools/ldlt_warm.py > gpurun_out/ldlt_warm.log 2>&1
