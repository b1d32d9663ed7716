# Iteration check: the whole -m gpu suite, a short bench line (no CPU legs, no scaled LBA), the
# config-4 LBA timing default vs dense-MFMA Schur, and an MFMA-Schur PMC pass.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -60 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 400 python -u bench.py --no-cpu --no-extras --no-lba-scaled > gpurun_out/bench.log 2>&1
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.log").read().strip().splitlines()[-1])
print("value", d["value"], "ms_per_step", d["ms_per_step"], "stages", d.get("stage_ms_per_batch"))
print("roofline", {k: d["roofline"].get(k) for k in ("achieved", "frac", "launch_ms", "algorithmic")})
print("pipeline_alg", d.get("pipeline_algorithmic"))
print("lba", d["lba"]["ms_per_iter"], d["lba"]["solve_ms"])
PY
timeout -k 10 120 python -u tools/lba_timing.py > gpurun_out/lbatime.log 2>&1; grep -E "median" gpurun_out/lbatime.log
ORB_LBA_SCHUR_MFMA=1 timeout -k 10 120 python -u tools/lba_timing.py > gpurun_out/lbatime.log 2>&1; grep -E "median" gpurun_out/lbatime.log
ORB_LBA_SCHUR_MFMA=1 bash tools/gpu_lba_pmc.sh c4_mfma
