#!/bin/bash
# Extraction profiles of the current tree (round 6): the isolated 256-frame launch's kernel stats
# (bench.py's roofline durations), the four PMC passes behind the roofline's traffic / VALU / lane
# figures, then one full default bench line -> gpurun_out/ (copied to profiles/r06_*).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
bash tools/gpu_ext_isolated.sh r06
bash tools/gpu_pmc_all.sh
cd $R
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.log 2>&1
tail -c 400 gpurun_out/bench_full.log
echo r6 prof ok
