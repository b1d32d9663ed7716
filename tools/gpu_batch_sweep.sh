#!/bin/bash
# Extraction step sweep (frames per step x streams), the bench's headline leg only, no stage events,
# three rounds interleaved -> gpurun_out/batch_sweep.txt
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
: > gpurun_out/batch_sweep.txt
for round in 1 2 3; do
  for cfg in "512 4" "1024 4" "1024 8" "768 6" "768 3"; do
    set -- $cfg
    v=$(timeout -k 10 120 python -u bench.py --no-cpu --no-lba --no-extras --no-stereo --no-profile --batch $1 --streams $2 --pool 1024 2>/dev/null | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
    echo "round $round batch $1 streams $2: $v" >> gpurun_out/batch_sweep.txt
  done
done
cat gpurun_out/batch_sweep.txt
