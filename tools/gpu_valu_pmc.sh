# VALU / issue PMC pass over the bench's extraction step (8 SQ + 2 GRBM counters, one pass)
# -> gpurun_out/pmc_valu, summarised into gpurun_out/valu_pmc.json by tools/pmc_valu.py.
set -e
R=$GRAFT_REPO_ROOT
bash $R/tools/pmc_run.sh valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_LDS \
    SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT
cd $R && python tools/pmc_valu.py gpurun_out/valu_pmc.json gpurun_out/pmc_valu width=640 height=480 nfeatures=1000 \
    frames_per_launch=128 > gpurun_out/valu_pmc.txt 2>&1
echo valu ok
