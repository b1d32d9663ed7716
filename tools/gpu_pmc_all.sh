# PMC passes for the bench's roofline (default bench configuration: 4 streams x 256 frames per
# launch): FETCH_SIZE, WRITE_SIZE (separate passes, MI355X_MICROARCH.md HBM section) and the VALU
# issue counters, the active-lane counter -> gpurun_out/pmc_traffic.json, gpurun_out/valu_pmc.json,
# gpurun_out/lanes_pmc.json (copied to profiles/rNN_*).
set -e
R=$GRAFT_REPO_ROOT
cd $R
bash tools/pmc_run.sh fetch FETCH_SIZE
bash tools/pmc_run.sh write WRITE_SIZE
bash tools/pmc_run.sh valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_LDS \
    SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT
bash tools/pmc_run.sh lanes SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE
cd $R
python tools/pmc_traffic.py gpurun_out/pmc_traffic.json fetch=gpurun_out/pmc_fetch write=gpurun_out/pmc_write \
    width=640 height=480 nfeatures=1000 frames_per_launch=256 streams=4 > gpurun_out/pmc_traffic.txt 2>&1
python tools/pmc_valu.py gpurun_out/valu_pmc.json gpurun_out/pmc_valu width=640 height=480 nfeatures=1000 \
    frames_per_launch=256 streams=4 > gpurun_out/valu_pmc.txt 2>&1
python tools/pmc_lanes.py gpurun_out/lanes_pmc.json gpurun_out/pmc_lanes width=640 height=480 nfeatures=1000 \
    frames_per_launch=256 streams=4 > gpurun_out/lanes_pmc.txt 2>&1
echo pmc all ok
