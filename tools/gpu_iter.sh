# Iteration run on the GPU box: the VALU issue-rate microbenchmark, the -m gpu tests selected by
# $1 (all when empty; every failure reported, the bench line runs regardless), then a short bench
# line (no CPU legs).  Outputs under gpurun_out/.
# Usage: gpurun -- bash tools/gpu_iter.sh ["pytest -k expression"]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -k "$K" > gpurun_out/gputest.log 2>&1
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/gputest.log 2>&1
fi
rc=$?
tail -5 gpurun_out/gputest.log
# a test run that ended on a GPU fault, an abort or a time limit ends the call here
case $rc in 0|1) ;; *) echo "pytest rc $rc: stopping"; exit $rc ;; esac
timeout -k 10 400 python -u bench.py --no-cpu --no-extras > gpurun_out/bench.log 2>&1 || exit $?
tail -c 600 gpurun_out/bench.log
exit $rc
