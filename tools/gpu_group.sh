# Device-side group exchange: group tests, the two-rank bench test, config-4 / 200 KF timing with the
# device exchange and with the host-ordered one, and a kernel trace of the device exchange.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_lba_group_gpu.py tests/test_bench_ranks.py tests/test_lba_gpu.py tests/test_cpp_shim.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/grptest.log 2>&1 || { tail -40 gpurun_out/grptest.log; exit 1; }
tail -2 gpurun_out/grptest.log
ORB_LBA_GROUP_DEVICE=1 timeout -k 10 150 python -u tools/lba_timing.py group=2 > gpurun_out/grp_c4.log 2>&1; tail -2 gpurun_out/grp_c4.log
ORB_LBA_GROUP_HOST=1 timeout -k 10 150 python -u tools/lba_timing.py group=2 > gpurun_out/grp_c4_host.log 2>&1; tail -2 gpurun_out/grp_c4_host.log
ORB_LBA_GROUP_DEVICE=1 timeout -k 10 200 python -u tools/lba_timing.py group=2 corridor=1 n_local=200 n_points=100000 > gpurun_out/grp_kf200.log 2>&1; tail -2 gpurun_out/grp_kf200.log
cd /tmp && ORB_LBA_GROUP_DEVICE=1 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_grp -o run -- python3 $GRAFT_REPO_ROOT/tools/lba_timing.py group=2 > $GRAFT_REPO_ROOT/gpurun_out/prof_grp.log 2>&1
cd $GRAFT_REPO_ROOT && python tools/kernel_stats.py gpurun_out/prof_grp/run_kernel_stats.csv "LBA config 4, lba_group of 2 contexts on one device (device-side exchange)" > gpurun_out/prof_grp_stats.txt; head -16 gpurun_out/prof_grp_stats.txt
