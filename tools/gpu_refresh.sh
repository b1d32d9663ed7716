# Round-end style refresh on the GPU box: smoke, full bench line, rocprofv3 stats of the bench,
# the LBA f64 MFMA PMC pass.  Outputs under gpurun_out/ (copied to profiles/ by hand).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.log 2>&1
bash tools/prof_run.sh
bash tools/gpu_lba_pmc.sh
echo refresh ok
