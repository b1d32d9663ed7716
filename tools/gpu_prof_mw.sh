set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 env ORB_LBA_NO_GRAPH=1 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_mw -o run -- python3 $R/tools/lba_timing.py corridor=1 n_local=200 n_points=100000 solves=3 > $R/gpurun_out/prof_mw.log 2>&1
f=$(find $R/gpurun_out/prof_mw -name "*kernel_stats.csv" | head -1)
python3 $R/tools/stats_summary.py $f $R/gpurun_out/prof_mw_stats.txt "200 KF fused mw"
head -30 $R/gpurun_out/prof_mw_stats.txt
