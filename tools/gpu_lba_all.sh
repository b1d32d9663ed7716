# every local-BA GPU test (single process, device group, torch.distributed ranks on one device)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_lba_gpu.py tests/test_global_ba.py tests/test_lba_dist_gpu.py tests/test_lba_group_gpu.py tests/test_cpp_shim_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lba_all.log 2>&1 || { tail -40 gpurun_out/lba_all.log; exit 1; }
tail -2 gpurun_out/lba_all.log
