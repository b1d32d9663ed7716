#!/bin/bash
# Round-6 profiles of the final sources: the isolated 256-frame extraction launch (roofline durations),
# the four extraction PMC passes, rocprofv3 kernel stats of a default bench run (extraction + LBA
# config 4 + config 5) and of the LBA windows -> gpurun_out/ (copied to profiles/r06_*).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
bash tools/gpu_ext_isolated.sh r06
bash tools/gpu_pmc_all.sh
cd $R
export TMPDIR=/tmp
bash tools/prof_run.sh --no-lba-scaled
python3 tools/kernel_stats.py gpurun_out/prof_bench/bench_kernel_stats.csv "bench.py default run (extraction 4 x 256 frames per step + LBA config 4 + config 5), round 6, four streams sharing the chip" > gpurun_out/bench_kernel_stats.txt
bash tools/gpu_lba_prof.sh
echo r6 profiles ok
