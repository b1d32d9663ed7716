set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="tests/test_sbp_kf.py tests/test_sbp_sim3.py tests/test_matcher_gpu.py"
ORB_SBP_SEQ_RESOLVE=1 timeout -k 10 300 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/sbp_seq.log 2>&1 || true
timeout -k 10 300 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/sbp_new.log 2>&1 || true
tail -8 gpurun_out/sbp_seq.log; tail -8 gpurun_out/sbp_new.log
timeout -k 10 300 python -u -m pytest tests/test_pose_gpu.py tests/test_cpp_shim_dropin.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pose_tests.log 2>&1 || { tail -30 gpurun_out/pose_tests.log; exit 1; }
tail -2 gpurun_out/pose_tests.log
bash tools/gpu_pose_timing.sh
