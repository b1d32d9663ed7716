# round-5 check: the reduced-solve harness, the matcher / pose tests touched by the pinned staging,
# and the routed-call latency rows.  Outputs under gpurun_out/.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_ldlt2.sh > /dev/null
timeout -k 5 120 tools/micro/valu_issue > gpurun_out/valu_issue.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_fuse.py tests/test_search_by_bow.py tests/test_triangulation.py tests/test_sim3_matcher.py tests/test_distinctive.py tests/test_pose_gpu.py tests/test_cpp_shim_loop.py tests/test_cpp_shim_dropin.py tests/test_extractor_gpu.py tests/test_bench_pipeline.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5a_tests.log 2>&1 || { tail -40 gpurun_out/r5a_tests.log; exit 1; }
tail -2 gpurun_out/r5a_tests.log
timeout -k 10 600 python -u tools/routed_calls.py > gpurun_out/routed.log 2>&1 || { tail -30 gpurun_out/routed.log; exit 1; }
bash tools/gpu_ab_multi.sh base 3 > gpurun_out/ab_octree.log 2>&1
cat gpurun_out/ab_octree.log
cat gpurun_out/ldlt2.log
cat gpurun_out/valu_issue.log
cat gpurun_out/routed.log
