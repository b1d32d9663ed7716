# round-5: reduced-solve clock split (timing variant) + the extraction step's stream gaps (kernel trace)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_ldlt_timing.sh
bash tools/prof_run.sh --no-lba --no-stereo --no-lba-scaled
python tools/ext_gap.py gpurun_out/prof_bench/bench_kernel_trace.csv > gpurun_out/ext_gap.txt 2>&1
python tools/ext_timeline.py gpurun_out/prof_bench/bench_kernel_trace.csv > gpurun_out/ext_timeline.txt 2>&1
cat gpurun_out/ext_gap.txt
head -12 gpurun_out/ext_timeline.txt
