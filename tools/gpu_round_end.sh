# Round-end refresh on the GPU box: the -m gpu suite, smoke, the full bench line.
# Outputs under gpurun_out/ (copied to profiles/ afterwards).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -60 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.log 2>&1
tail -c 400 gpurun_out/bench_full.log
echo round-end ok
