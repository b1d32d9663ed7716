# LBA iteration loop on the GPU box: parity tests, the ORB_TIMING clock split, a bench line.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lba_gpu.py tests/test_lba_dist_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/lba_tests.log 2>&1
ORB_SLAM2_AMD_LIB=$PWD/orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so timeout -k 10 120 python -u tools/lba_timing.py > gpurun_out/lba_timing.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --no-extras --steps 5 --warmup 2 > gpurun_out/bench_lba.log 2>&1
echo ok
