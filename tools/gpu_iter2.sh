# LBA iteration: lba tests, config-4 timing default vs dense-MFMA Schur (+ its kernel times), and
# the ORB_TIMING clock split of k_ldlt_solve (n = 114) from the variant build.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_lba_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lbatest.log 2>&1 || { tail -40 gpurun_out/lbatest.log; exit 1; }
tail -2 gpurun_out/lbatest.log
timeout -k 10 120 python -u tools/lba_timing.py > gpurun_out/lbatime.log 2>&1; grep -E "median" gpurun_out/lbatime.log
ORB_LBA_SCHUR_MFMA=1 timeout -k 10 120 python -u tools/lba_timing.py > gpurun_out/lbatime.log 2>&1; grep -E "median" gpurun_out/lbatime.log
cd /tmp && ORB_LBA_SCHUR_MFMA=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_mfma -o run -- python3 $GRAFT_REPO_ROOT/tools/lba_timing.py > $GRAFT_REPO_ROOT/gpurun_out/prof_mfma.log 2>&1
cd $GRAFT_REPO_ROOT && python tools/kernel_stats.py gpurun_out/prof_mfma/run_kernel_stats.csv "MFMA Schur" > gpurun_out/prof_mfma.txt; head -12 gpurun_out/prof_mfma.txt
ORB_SLAM2_AMD_LIB=$GRAFT_REPO_ROOT/orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so timeout -k 10 60 python -u tools/ldlt_warm.py > gpurun_out/ldlt_timing.log 2>&1; tail -4 gpurun_out/ldlt_timing.log
