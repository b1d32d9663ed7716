set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lba_gpu.py tests/test_lba_group_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lbatest.log 2>&1 || { tail -40 gpurun_out/lbatest.log; exit 1; }
tail -2 gpurun_out/lbatest.log
for a in "" "corridor=1 n_local=60 n_points=8000" "corridor=1 n_local=200 n_points=100000"; do
  timeout -k 10 300 python -u tools/lba_timing.py $a > gpurun_out/lbatime.log 2>&1; grep -E "problem|median" gpurun_out/lbatime.log
done
ORB_LBA_SCHUR_MFMA=1 timeout -k 10 120 python -u tools/lba_timing.py > gpurun_out/lbatime.log 2>&1; grep -E "median" gpurun_out/lbatime.log
bash tools/gpu_lba_prof.sh
