# extraction-leg throughput over (frames per step, streams): bench.py's extraction leg only
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "512 4" "512 8" "1024 4" "1024 8" "768 6" "512 4"; do
  set -- $cfg
  timeout -k 10 150 python -u bench.py --steps 30 --warmup 5 --batch $1 --streams $2 --no-cpu --no-profile --no-lba --no-extras > gpurun_out/sweep_$1_$2.json 2> gpurun_out/sweep_$1_$2.err
  python - $1 $2 <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/sweep_{sys.argv[1]}_{sys.argv[2]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], sys.argv[2], round(d["value"]), d["ms_per_step"])
PY
done
