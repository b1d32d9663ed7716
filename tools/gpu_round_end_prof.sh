# Round-end profiles: rocprofv3 kernel stats of the bench, the LBA kernel stats (config 4, 60 KF,
# 200 KF), the LBA f64 MFMA PMC passes (default and dense-MFMA Schur), lba_group timing.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/prof_run.sh --no-lba-scaled
python tools/kernel_stats.py gpurun_out/prof_bench/bench_kernel_stats.csv "bench.py default run (extraction + LBA config 4 + config 5)" > gpurun_out/bench_kernel_stats.txt
python tools/ext_timeline.py gpurun_out/prof_bench/bench_kernel_trace.csv > gpurun_out/ext_timeline.txt 2>&1
bash tools/gpu_lba_prof.sh
bash tools/gpu_lba_pmc.sh c4
ORB_LBA_SCHUR_MFMA=1 bash tools/gpu_lba_pmc.sh c4_mfma
timeout -k 10 150 python tools/lba_timing.py group=2 > gpurun_out/grp_c4.log 2>&1
timeout -k 10 200 python tools/lba_timing.py group=2 corridor=1 n_local=200 n_points=100000 > gpurun_out/grp_kf200.log 2>&1
tail -1 gpurun_out/grp_c4.log; tail -1 gpurun_out/grp_kf200.log
echo prof ok
