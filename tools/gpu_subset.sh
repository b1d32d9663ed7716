set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_cpp_shim_dropin.py tests/test_lba_dist_gpu.py tests/test_lba_group_gpu.py tests/test_bench_ranks.py tests/test_abi.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/g1.log 2>&1 || { tail -60 gpurun_out/g1.log; exit 1; }
tail -5 gpurun_out/g1.log
