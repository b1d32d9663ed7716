# Full default bench line (N=1) + rocprofv3 kernel stats of the bench's extraction / LBA legs.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
bash tools/prof_run.sh
