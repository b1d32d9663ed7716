#!/bin/bash
# The bench's own 256-frame extraction launch alone on one stream (bench.py --streams 1 --batch 256:
# every kernel serialised, nothing sharing the chip) under rocprofv3 --kernel-trace --stats ->
# gpurun_out/ext_isolated_stats.txt (copied to profiles/rNN_ext_isolated_stats.txt; bench.py's
# roofline reads the per-kernel average durations from that file).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06}
export TMPDIR=/tmp
cd /tmp
rm -rf $R/gpurun_out/prof_iso
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_iso -o iso -- \
    python3 $R/bench.py --streams 1 --batch 256 --steps 20 --warmup 5 --no-cpu --no-lba --no-extras --no-stereo \
    --no-profile > $R/gpurun_out/prof_iso.log 2>&1
cd $R
CSV=$(find gpurun_out/prof_iso -name 'iso_kernel_stats.csv' -print -quit)
{
  python3 tools/kernel_stats.py "$CSV" "bench.py --streams 1 --batch 256 --steps 20 --warmup 5 --no-cpu --no-lba" \
      "--no-extras --no-stereo --no-profile: one 256-frame extraction launch + SearchForInitialization per step (frames_per_launch=256)," \
      "alone on one HIP stream (kernels serialised), $TAG"
  echo "provenance $(python3 tools/pmc_provenance.py | tr -d '\n ')"
  echo "bench line: $( (grep "^{\"metric" gpurun_out/prof_iso.log || true) | tail -1 | cut -c1-300)"
} > gpurun_out/ext_isolated_stats.txt
cat gpurun_out/ext_isolated_stats.txt | head -14
