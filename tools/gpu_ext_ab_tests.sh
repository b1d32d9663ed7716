# extraction GPU tests (bit-exact against the oracle), then the same-box A/B of variant $1 against the tree
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_bench_pipeline.py tests/test_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ext_tests.log 2>&1 || { tail -40 gpurun_out/ext_tests.log; exit 1; }
tail -1 gpurun_out/ext_tests.log
bash tools/gpu_ab_ext.sh ${1:-base} ${2:-3}
