# Round-3 measurement pack: lba_group exchange latency (two contexts on device 0), f64 MFMA / VALU
# PMC passes of the local BA (config 4 default and dense-MFMA Schur; 60 KF corridor), and the
# extraction kernels' active-lane counter (SQ_THREAD_CYCLES_VALU).  Outputs under gpurun_out/.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
timeout -k 10 150 python tools/lba_timing.py group=2 > gpurun_out/grp_c4.log 2>&1
timeout -k 10 200 python tools/lba_timing.py group=2 corridor=1 n_local=200 n_points=100000 > gpurun_out/grp_kf200.log 2>&1
bash tools/gpu_lba_pmc.sh c4
ORB_LBA_SCHUR_MFMA=1 bash tools/gpu_lba_pmc.sh c4_mfma
ORB_LBA_NO_GRAPH=1 bash tools/gpu_lba_pmc.sh kf60 corridor=1 n_local=60 n_points=8000
bash tools/pmc_run.sh lanes SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE
python tools/pmc_lanes.py gpurun_out/lanes_pmc.json gpurun_out/pmc_lanes width=640 height=480 nfeatures=1000 frames_per_launch=128 > gpurun_out/lanes_pmc.txt 2>&1
echo measure ok
