# local-BA GPU tests, the dataflow solve's ORB_TIMING split, then the same-box A/B of variant base
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lba_gpu.py tests/test_global_ba.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lba_tests.log 2>&1 || { tail -40 gpurun_out/lba_tests.log; exit 1; }
tail -1 gpurun_out/lba_tests.log
bash tools/gpu_ldlt_timing.sh
bash tools/gpu_ab_lba.sh base ${1:-2}
