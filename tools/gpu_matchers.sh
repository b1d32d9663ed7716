# matcher / projection-search GPU tests, the routed-call latency rows, and the VALU issue micro
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_matcher_gpu.py tests/test_sbp_kf.py tests/test_sbp_sim3.py tests/test_search_by_bow.py tests/test_fuse.py tests/test_sim3_matcher.py tests/test_triangulation.py tests/test_cpp_shim.py tests/test_cpp_shim_dropin.py tests/test_abi.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/m_tests.log 2>&1 || { tail -60 gpurun_out/m_tests.log; exit 1; }
tail -3 gpurun_out/m_tests.log
timeout -k 10 300 python -u tools/routed_calls.py > gpurun_out/routed.log 2>&1 || { tail -30 gpurun_out/routed.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_pose_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pose_tests.log 2>&1 || { tail -30 gpurun_out/pose_tests.log; exit 1; }
tail -1 gpurun_out/pose_tests.log
