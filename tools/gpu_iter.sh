# Iteration run on the GPU box: the VALU issue-rate microbenchmark, the -m gpu tests selected by
# $1 (all when empty), then a short bench line (no CPU legs).  Outputs under gpurun_out/.
# Usage: gpurun -- bash tools/gpu_iter.sh ["pytest -k expression"]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -x tools/micro/valu_issue ]; then
  timeout -k 10 120 tools/micro/valu_issue > gpurun_out/valu_issue.txt 2>&1
  cat gpurun_out/valu_issue.txt
fi
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "$K" > gpurun_out/gputest.log 2>&1 || { tail -60 gpurun_out/gputest.log; exit 1; }
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -60 gpurun_out/gputest.log; exit 1; }
fi
tail -3 gpurun_out/gputest.log
timeout -k 10 400 python -u bench.py --no-cpu --no-extras > gpurun_out/bench.log 2>&1
tail -c 1500 gpurun_out/bench.log
