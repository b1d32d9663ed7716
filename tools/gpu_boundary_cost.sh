# Cost of one kernel boundary inside the LM slot graphs: config-4 timing with and without four
# extra empty launches per slot (ORB_LBA_EXTRA_BOUNDARY), alternated on one box.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3; do
timeout -k 10 120 python -u tools/lba_timing.py > gpurun_out/bc.log 2>&1; echo "default $(grep median gpurun_out/bc.log)"
ORB_LBA_EXTRA_BOUNDARY=1 timeout -k 10 120 python -u tools/lba_timing.py > gpurun_out/bc.log 2>&1; echo "extra4 $(grep median gpurun_out/bc.log)"
done
