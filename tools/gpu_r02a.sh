# round-2 first measurement: bench (N=1, then 2 ranks on the one GPU), kernel stats, VALU PMC
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full.log 2>&1
timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 3 --no-extras > gpurun_out/bench2.log 2>&1
bash tools/prof_run.sh
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1) || true
bash tools/gpu_valu_pmc.sh
echo r02a ok
