set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_extractor_gpu.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ext.log 2>&1
timeout -k 10 120 python -u bench.py --no-cpu --no-lba --no-extras --no-stereo > gpurun_out/bench_q.log 2>&1
bash tools/gpu_pmc_all.sh
timeout -k 10 120 python -u bench.py --no-cpu --no-lba --no-extras --no-stereo > gpurun_out/bench_q2.log 2>&1
echo ok
