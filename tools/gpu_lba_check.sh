# LBA parity tests, solve times (tools/lba_timing.py medians, three runs), rocprofv3 kernel stats
set -e
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_lba_gpu.py tests/test_global_ba.py tests/test_lba_dist_gpu.py tests/test_cpp_shim.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lba_tests.log 2>&1
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/lba_timing.py 2>&1 | tail -1 >> gpurun_out/lba_cmp.log
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_lba6 -o lba -- python3 $R/tools/lba_timing.py > $R/gpurun_out/prof_lba6.log 2>&1
cd $R && python tools/stats_summary.py gpurun_out/prof_lba6/lba_kernel_stats.csv gpurun_out/lba_stats.txt "rocprofv3 --kernel-trace --stats -- python3 tools/lba_timing.py" 
echo ok
