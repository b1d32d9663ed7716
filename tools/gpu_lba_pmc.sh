# f64 MFMA / VALU PMC pass over the local-BA solves -> gpurun_out/pmc_lba (one pass: 6 SQ + 1 GRBM counters)
set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_lba -o run -- python3 $R/tools/lba_timing.py > $R/gpurun_out/pmc_lba.log 2>&1
cd $R && python tools/pmc_lba.py gpurun_out/lba_pmc.json gpurun_out/pmc_lba > gpurun_out/lba_pmc.txt 2>&1
echo ok
