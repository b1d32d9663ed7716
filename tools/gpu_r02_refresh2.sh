# Round-2 refresh after the LBA changes: smoke, the default bench line, rocprofv3 kernel stats of
# the bench and of the local-BA solves, the f64 MFMA PMC pass over the solves.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
bash tools/prof_run.sh
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_lba -o lba -- python3 $GRAFT_REPO_ROOT/tools/lba_timing.py > $GRAFT_REPO_ROOT/gpurun_out/prof_lba.log 2>&1
cd $GRAFT_REPO_ROOT && bash tools/gpu_lba_pmc.sh
echo refresh ok
