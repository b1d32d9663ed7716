# A short bench line without the CPU legs (checks the line's fields after a bench.py change).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --no-cpu --no-extras > gpurun_out/bench_quick.log 2>&1
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench_quick.log") if l.startswith("{")][-1])
print("value", d["value"], "lba", d["lba"]["ms_per_iter"])
print(json.dumps(d.get("lba_scaled"))[:1500])
PY
