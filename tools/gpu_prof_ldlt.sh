# rocprofv3 kernel stats of config-4 local BA with the old and the dataflow reduced solve (slot graphs)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for which in old df; do
  if [ $which = old ]; then E="ORB_LBA_LDLT_OLD=1"; else E="ORB_LBA_X=0"; fi
  timeout -k 10 300 env $E rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_ldlt_$which -o run -- python3 $R/tools/lba_timing.py > $R/gpurun_out/prof_ldlt_$which.log 2>&1
  f=$(find $R/gpurun_out/prof_ldlt_$which -name "*kernel_stats.csv" | head -1)
  python3 $R/tools/stats_summary.py $f $R/gpurun_out/prof_ldlt_${which}_stats.txt "LBA config 4, reduced solve $which"
  grep median $R/gpurun_out/prof_ldlt_$which.log
  head -12 $R/gpurun_out/prof_ldlt_${which}_stats.txt
done
