#!/bin/bash
# LocalBundleAdjustment through the compiled drop-in (shim_caller timeit) on the config-4 window:
# per-call median and the phase medians (gather, arrays, lba_solve, write-back), GPU solve and the
# like-for-like CPU column (the same shim around the oracle's solve), at ORB_SHIM_THREADS = 0 / 4 / 8
# host pool workers -> gpurun_out/shim_lba_phases.txt
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
python3 tools/mk_lba_in.py gpurun_out/lba_c4.in
{
  for t in 0 4 8; do
    echo "threads $t gpu: $(ORB_SHIM_THREADS=$t timeout -k 10 120 orb-slam2-_amd/lib/shim_caller timeit 20 lba gpurun_out/lba_c4.in)"
  done
  for t in 0 4; do
    echo "threads $t cpu: $(ORB_SHIM_THREADS=$t ORB_ORACLE_LIB=$R/oracle/build/liborb_oracle.so timeout -k 10 300 orb-slam2-_amd/lib/shim_caller timeit 5 lbacpu gpurun_out/lba_c4.in)"
  done
} > gpurun_out/shim_lba_phases.txt
cat gpurun_out/shim_lba_phases.txt
