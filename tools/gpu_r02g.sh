set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_extractor_gpu.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ext.log 2>&1
ORB_SLAM2_AMD_LIB=orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so timeout -k 10 120 python -u tools/fast_timing.py > gpurun_out/timing.log 2>&1
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_1s -o bench -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 20 --warmup 5 --no-lba --no-extras --no-stereo --streams 1 --batch 64 > $GRAFT_REPO_ROOT/gpurun_out/prof_1s.log 2>&1
cd $GRAFT_REPO_ROOT
for a in "" "--streams 2 --batch 256"; do
  echo "== $a" >> gpurun_out/sweep3.log
  timeout -k 10 120 python -u bench.py --no-cpu --no-lba --no-extras --no-stereo $a 2>&1 | tail -1 | cut -c1-120 >> gpurun_out/sweep3.log
done
echo ok
