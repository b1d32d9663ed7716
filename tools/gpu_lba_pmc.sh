# f64 MFMA / VALU PMC pass over the local-BA solves -> gpurun_out/pmc_lba_TAG (one pass: 6 SQ + 1 GRBM counters)
# usage: tools/gpu_lba_pmc.sh TAG [lba_timing.py args...]; library switches (ORB_LBA_SCHUR_MFMA, ORB_LBA_NO_GRAPH)
# pass through the environment.
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-c4}; shift || true
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_lba_$TAG -o run -- python3 $R/tools/lba_timing.py "$@" > $R/gpurun_out/pmc_lba_$TAG.log 2>&1
cd $R && python tools/pmc_lba.py gpurun_out/lba_pmc_$TAG.json gpurun_out/pmc_lba_$TAG "$@" > gpurun_out/lba_pmc_$TAG.txt 2>&1
echo ok $TAG
