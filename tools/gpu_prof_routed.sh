# kernel-level profile of the routed-call latency rows (per-kernel averages under rocprofv3)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_routed -o run -- python3 $GRAFT_REPO_ROOT/tools/routed_calls.py --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof_routed.log 2>&1
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/prof_routed -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/prof_routed_stats.csv
head -40 gpurun_out/prof_routed_stats.csv | cut -d, -f1-8
