# rocprofv3 kernel statistics of the 200 KF corridor solve (kernels one by one), at the given
# ORB_LBA_SMALL_PAIR thresholds (k_schur_pairs' wave / workgroup split)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for sp in ${1:-512}; do
  timeout -k 10 300 env ORB_LBA_NO_GRAPH=1 ORB_LBA_SMALL_PAIR=$sp rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_kf200_$sp -o run -- python3 $R/tools/lba_timing.py corridor=1 n_local=200 n_points=100000 > $R/gpurun_out/prof_kf200_$sp.log 2>&1
  f=$(find $R/gpurun_out/prof_kf200_$sp -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] || { tail -5 $R/gpurun_out/prof_kf200_$sp.log; exit 1; }
  python3 $R/tools/stats_summary.py $f $R/gpurun_out/prof_kf200_${sp}_stats.txt "LBA corridor 200 KF x 100k, kernels one by one, ORB_LBA_SMALL_PAIR=$sp"
  echo "== small-pair threshold $sp"; grep median $R/gpurun_out/prof_kf200_$sp.log
  head -12 $R/gpurun_out/prof_kf200_${sp}_stats.txt | tail -9
done
