set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_2s -o bench -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 20 --warmup 5 --no-lba --no-extras --no-stereo --no-profile > $GRAFT_REPO_ROOT/gpurun_out/prof_2s.log 2>&1
echo ok
