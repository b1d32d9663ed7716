# extraction-leg throughput with per-sequence HIP stream priorities (ORB_BENCH_STREAM_PRIO), interleaved.
# The switch lived in bench.py (SequencePipeline: torch.cuda.Stream(dev, priority=...)) for the round-5
# measurement only (6-9 % slower) and was removed; re-add it there to repeat the run.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for r in 1 2; do
for pr in "0" "-1,0,0,0" "-1,-1,0,0" "0,-1,0,-1"; do
  ORB_BENCH_STREAM_PRIO=$pr timeout -k 10 150 python -u bench.py --steps 30 --warmup 5 --no-cpu --no-profile --no-lba --no-extras --no-stereo > gpurun_out/prio.json 2> gpurun_out/prio.err
  python -c "
import json; d=json.loads(open('gpurun_out/prio.json').read().strip().splitlines()[-1]); print('$pr', round(d['value']), d['ms_per_step'])"
done
done
