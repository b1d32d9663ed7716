# Full GPU test suite, smoke and the default bench line on the current tree.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo check ok
