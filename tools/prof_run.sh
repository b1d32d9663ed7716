#!/bin/bash
# rocprofv3 kernel-trace summaries of bench.py (extraction step and local BA) -> gpurun_out/prof_*
# usage: tools/prof_run.sh [extra bench.py args]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o bench -- \
    python3 $R/bench.py --no-cpu --steps 20 --warmup 5 --lba-solves 5 --no-extras "$@" > $R/gpurun_out/prof_bench.log 2>&1
echo prof done
