#!/bin/bash
# Same-box A/B of the extraction step with the isolated per-kernel durations: a library variant
# (ORB_SLAM2_AMD_LIB) against the default build, alternating, bench.py's default step (stage events
# only after the timed region) without the CPU / LBA / stereo / extras legs.
# usage: gpu_ab_ext2.sh VARIANT_NAME [rounds]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/orb-slam2-_amd/lib/variant/$1/liborbslam2_amd.so
for i in $(seq ${2:-3}); do
  for which in variant default; do
    if [ $which = variant ]; then export ORB_SLAM2_AMD_LIB=$V; else unset ORB_SLAM2_AMD_LIB; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-lba --no-stereo --no-extras --steps 20 --warmup 5 > gpurun_out/ab.log 2>&1
    python -c "import json; d=json.loads([l for l in open('gpurun_out/ab.log') if l.startswith('{')][-1]); print('$which', d['value'], d['ms_per_step'], d.get('stage_ms_isolated_live'))"
  done
done
