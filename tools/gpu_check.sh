# GPU check used while iterating: the whole -m gpu suite, then a short bench line (no CPU legs).
# Usage: gpurun -- bash tools/gpu_check.sh [pytest -k expression]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/gputest.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
fi
tail -3 gpurun_out/gputest.log
timeout -k 10 400 python -u bench.py --no-cpu --no-extras > gpurun_out/bench.log 2>&1
tail -c 3000 gpurun_out/bench.log
