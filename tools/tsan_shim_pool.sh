#!/bin/bash
# ThreadSanitizer run of the drop-in LocalBundleAdjustment's host pool (include/orbslam2_amd_shim.hpp:
# HostPool, the parallel gather / arrays / write-back): the compiled caller built with
# -fsanitize=thread, mode lbacpu (the oracle's solve, no GPU needed) on the config-4 window, 4 pool
# workers, several calls through one thread's pool.  Runs in the build container.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
g++ -std=c++17 -O1 -g -fsanitize=thread -ffp-contract=off -pthread -I$R/include $R/tests/cpp/shim_caller.cpp \
    -L$R/orb-slam2-_amd/lib -lorbslam2_amd -ldl -Wl,-rpath,$R/orb-slam2-_amd/lib -o $T/sc_tsan
python3 $R/tools/mk_lba_in.py $T/lba.in
ORB_SHIM_THREADS=4 ORB_ORACLE_LIB=$R/oracle/build/liborb_oracle.so TSAN_OPTIONS="halt_on_error=1" \
    $T/sc_tsan timeit 3 lbacpu $T/lba.in
echo "tsan shim pool ok (no ThreadSanitizer report in 6 calls)"
rm -rf $T
