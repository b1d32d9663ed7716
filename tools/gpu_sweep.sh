# Extraction step sweep: streams x frames per launch (bench.py --batch = streams x frames).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "3 384" "4 512" "4 384" "2 384" "3 480" "6 384"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --no-cpu --no-lba --no-stereo --no-extras --no-profile --streams $1 --batch $2 --steps 30 --warmup 5 > gpurun_out/sweep.log 2>&1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/sweep.log') if l.startswith('{')][-1]); print('streams $1 batch $2', d['value'], d['ms_per_step'])"
done
