cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K="test_search_by_projection_kf_gpu or test_search_for_initialization"
timeout -k 10 200 python -u -m pytest tests/test_sbp_kf.py tests/test_matcher_gpu.py -k "$K" -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/ab_cur.log 2>&1; echo "cur rc $?"
ORB_SLAM2_AMD_LIB=$GRAFT_REPO_ROOT/orb-slam2-_amd/lib/variant/prestage/liborbslam2_amd.so timeout -k 10 200 python -u -m pytest tests/test_sbp_kf.py tests/test_matcher_gpu.py -k "$K" -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/ab_pre.log 2>&1; echo "prestage rc $?"
grep -h "passed\|failed\|Abort\|free()" gpurun_out/ab_cur.log gpurun_out/ab_pre.log | head
