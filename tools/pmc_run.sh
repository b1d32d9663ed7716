#!/bin/bash
# One rocprofv3 PMC pass (counters given as arguments) over a short bench.py run -> gpurun_out/pmc_<tag>
# usage: tools/pmc_run.sh TAG COUNTER... ; counters only with --kernel-trace (no sys/runtime traces).
# Extra bench.py arguments can be passed in $PMC_BENCH_ARGS; the default is the bench's own
# configuration (4 streams x 256 frames per launch) so per-launch counters match bench.py's roofline.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $R/gpurun_out/pmc_$TAG -o run -- \
    python3 $R/bench.py --no-cpu --no-lba --no-extras --no-stereo --steps 5 --warmup 2 $PMC_BENCH_ARGS > $R/gpurun_out/pmc_$TAG.log 2>&1
echo pmc done
