# LBA parity tests, then solve times: device-built structure (default) vs the host build
set -e
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_lba_gpu.py tests/test_global_ba.py tests/test_lba_dist_gpu.py tests/test_cpp_shim.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lba_tests.log 2>&1
for i in 1 2; do
  echo "== device structure" >> gpurun_out/lba_cmp.log
  timeout -k 10 120 python -u tools/lba_timing.py 2>&1 | tail -1 >> gpurun_out/lba_cmp.log
  echo "== host structure" >> gpurun_out/lba_cmp.log
  ORB_LBA_HOST_STRUCT=1 timeout -k 10 120 python -u tools/lba_timing.py 2>&1 | tail -1 >> gpurun_out/lba_cmp.log
done
echo ok
