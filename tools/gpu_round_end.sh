# Round-end refresh on the GPU box: smoke, the full bench line, rocprofv3 kernel stats of the
# bench, the FETCH_SIZE / WRITE_SIZE passes for the roofline traffic, the LBA f64 MFMA PMC pass.
# Outputs under gpurun_out/ (copied to profiles/ afterwards).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.log 2>&1
bash tools/prof_run.sh
bash tools/pmc_run.sh fetch FETCH_SIZE
bash tools/pmc_run.sh write WRITE_SIZE
bash tools/gpu_lba_pmc.sh
echo round-end ok
