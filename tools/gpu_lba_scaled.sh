set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_lba_gpu.py tests/test_global_ba.py tests/test_lba_dist_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/lbatest.log 2>&1 || { tail -30 gpurun_out/lbatest.log; exit 1; }
tail -3 gpurun_out/lbatest.log
for a in "" "corridor=1 n_local=60 n_points=8000" "corridor=1 n_local=200 n_points=100000"; do
  timeout -k 10 300 python -u tools/lba_timing.py $a > gpurun_out/lbatime.log 2>&1; grep -E "problem|median" gpurun_out/lbatime.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof200 -o run -- python3 $GRAFT_REPO_ROOT/tools/lba_timing.py corridor=1 n_local=200 n_points=100000 > $GRAFT_REPO_ROOT/gpurun_out/prof200.log 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/prof200 -name "*kernel_stats.csv" | head -1 | xargs -I{} python3 $GRAFT_REPO_ROOT/tools/stats_summary.py {} $GRAFT_REPO_ROOT/gpurun_out/prof200_stats.txt "LBA 200 KF x 100k corridor"
head -30 $GRAFT_REPO_ROOT/gpurun_out/prof200_stats.txt
