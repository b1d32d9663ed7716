# rocprofv3 kernel statistics of the local-BA solves: config 4 (graphs, as timed) and the scaled
# corridor windows (60 KF x 8000, 200 KF x 100k points; ORB_LBA_NO_GRAPH: kernels enqueued one by
# one, rocprofv3 has crashed instrumenting the 2,500-node slot graphs of the 200 KF window)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
prof() {   # name, env, args
  timeout -k 10 300 env $2 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$1 -o run -- python3 $R/tools/lba_timing.py $3 > $R/gpurun_out/prof_$1.log 2>&1
  f=$(find $R/gpurun_out/prof_$1 -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] || { tail -5 $R/gpurun_out/prof_$1.log; exit 1; }
  python3 $R/tools/stats_summary.py $f $R/gpurun_out/prof_$1_stats.txt "$4"
  grep median $R/gpurun_out/prof_$1.log
  head -14 $R/gpurun_out/prof_$1_stats.txt
}
prof c4 "ORB_LBA_X=0" "" "LBA config 4 (20 KF x 3000), slot graphs"
prof kf60 "ORB_LBA_NO_GRAPH=1" "corridor=1 n_local=60 n_points=8000" "LBA corridor 60 KF x 8000, kernels one by one"
prof kf200 "ORB_LBA_NO_GRAPH=1" "corridor=1 n_local=200 n_points=100000" "LBA corridor 200 KF x 100k, kernels one by one"
