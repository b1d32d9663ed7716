set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_matcher_gpu.py tests/test_golden.py tests/test_abi.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_m.log 2>&1
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_1s -o bench -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 20 --warmup 5 --no-lba --no-extras --no-stereo --streams 1 --batch 64 --no-match-stream > $GRAFT_REPO_ROOT/gpurun_out/prof_1s.log 2>&1
cd $GRAFT_REPO_ROOT
for a in "--no-match-stream" "" "--streams 2 --batch 256 --no-match-stream"; do
  echo "== $a" >> gpurun_out/sweep2.log
  timeout -k 10 120 python -u bench.py --no-cpu --no-lba --no-extras --no-stereo $a 2>&1 | tail -1 | cut -c1-120 >> gpurun_out/sweep2.log
done
echo ok
