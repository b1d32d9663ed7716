# Extraction-step kernel trace (bench configuration, no LBA / stereo / CPU legs) for tools/ext_timeline.py.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/prof_run.sh --no-lba --no-stereo
python tools/ext_timeline.py gpurun_out/prof_bench/bench_kernel_trace.csv > gpurun_out/ext_timeline.txt 2>&1
cat gpurun_out/ext_timeline.txt
tail -c 600 gpurun_out/prof_bench.log
