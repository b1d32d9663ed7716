set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
A="--steps 2 --warmup 1 --batch 8 --streams 1 --pool 16 --no-cpu --no-lba-scaled --no-extras --no-profile --lba-solves 1 --lba-points 1500 --stereo-batches 2"
echo start > gpurun_out/dbg_progress.log
BENCH_STACKS_AFTER=40 timeout -k 10 100 python -u bench.py --gpus 1 $A > gpurun_out/dbg1.log 2>&1 || { echo "n1 rc=$?"; tail -60 gpurun_out/dbg1.log; exit 1; }
echo n1 ok >> gpurun_out/dbg_progress.log
BENCH_STACKS_AFTER=40 timeout -k 10 120 python -u bench.py --gpus 2 $A > gpurun_out/dbg2.log 2>&1 || { echo "n2 rc=$?"; tail -80 gpurun_out/dbg2.log; exit 1; }
echo n2 ok
