# LBA iteration loop: lba + group + global-BA tests, config-4 / 60 KF timing, k_ldlt_solve clock split (ORB_TIMING variant), config-4 kernel stats.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_lba_gpu.py tests/test_lba_group_gpu.py tests/test_global_ba.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lbatest.log 2>&1 || { tail -40 gpurun_out/lbatest.log; exit 1; }
tail -2 gpurun_out/lbatest.log
for a in "" "corridor=1 n_local=60 n_points=8000" "corridor=1 n_local=200 n_points=100000"; do
  timeout -k 10 200 python -u tools/lba_timing.py $a > gpurun_out/lbatime.log 2>&1; grep -E "median" gpurun_out/lbatime.log
done
ORB_SLAM2_AMD_LIB=$GRAFT_REPO_ROOT/orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so timeout -k 10 60 python -u tools/ldlt_warm.py > gpurun_out/ldlt_timing.log 2>&1; tail -4 gpurun_out/ldlt_timing.log
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -o run -- python3 $GRAFT_REPO_ROOT/tools/lba_timing.py > $GRAFT_REPO_ROOT/gpurun_out/prof_c4.log 2>&1
cd $GRAFT_REPO_ROOT && python tools/kernel_stats.py gpurun_out/prof_c4/run_kernel_stats.csv "LBA config 4" > gpurun_out/prof_c4_stats.txt; head -10 gpurun_out/prof_c4_stats.txt
