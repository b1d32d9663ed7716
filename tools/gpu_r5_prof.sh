# Round-5 profiles: rocprofv3 kernel stats of the bench run, then the PMC passes (traffic, VALU,
# lanes) of the bench's extraction configuration, each step under its own time limit.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
bash tools/prof_run.sh
python tools/kernel_stats.py gpurun_out/prof_bench/bench_kernel_stats.csv "bench.py default run (extraction + LBA config 4 + config 5), round 5" > gpurun_out/bench_kernel_stats.txt
python tools/ext_timeline.py gpurun_out/prof_bench/bench_kernel_trace.csv > gpurun_out/ext_timeline.txt 2>&1 || true
python tools/ext_gap.py gpurun_out/prof_bench/bench_kernel_trace.csv > gpurun_out/ext_gap.txt 2>&1 || true
bash tools/gpu_pmc_all.sh
echo r5 prof ok
