# LBA: solve time against the number of LM slots per captured graph (ORB_LBA_GRAPH_SLOTS),
# then a rocprofv3 kernel trace at the default for the gap timeline
set -e
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for n in 100 10 5 3; do
  echo "== slots per graph $n" >> gpurun_out/lba_chunks.log
  ORB_LBA_GRAPH_SLOTS=$n timeout -k 10 120 python -u tools/lba_timing.py 2>&1 | tail -1 >> gpurun_out/lba_chunks.log
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_lba5 -o lba -- python3 $R/tools/lba_timing.py > $R/gpurun_out/prof_lba5.log 2>&1
cd $R && python tools/lba_trace.py gpurun_out/prof_lba5/lba_kernel_trace.csv > gpurun_out/lba_trace5.txt 2>&1
echo ok
