set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
for b in 1 8 64 256; do timeout -k 10 300 python bench.py --no-cpu --batch $b --steps 10 --warmup 3 >> gpurun_out/bench_b.log 2>&1; done
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 > $R/gpurun_out/prof.log 2>&1
echo done
