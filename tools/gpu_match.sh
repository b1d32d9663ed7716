set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_matcher_gpu.py tests/test_extractor_gpu.py tests/test_cpp_shim.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_match.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --no-lba --no-extras --no-stereo > gpurun_out/bench_m.json 2> gpurun_out/bench_m.err
