# A/B of a library variant (tools/build_variant.py NAME ...): the LBA tests and config-4 timing with
# the variant, then the default build's timing.  usage: gpu_ab_variant.sh NAME
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/orb-slam2-_amd/lib/variant/$1/liborbslam2_amd.so
ORB_SLAM2_AMD_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_lba_gpu.py tests/test_global_ba.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_test.log 2>&1 || { tail -30 gpurun_out/ab_test.log; exit 1; }
tail -1 gpurun_out/ab_test.log
for i in 1 2; do
ORB_SLAM2_AMD_LIB=$V timeout -k 10 120 python -u tools/lba_timing.py > gpurun_out/ab_t.log 2>&1; echo "variant $(grep median gpurun_out/ab_t.log)"
timeout -k 10 120 python -u tools/lba_timing.py > gpurun_out/ab_t.log 2>&1; echo "default $(grep median gpurun_out/ab_t.log)"
done
