# The CPU side under AddressSanitizer + UndefinedBehaviorSanitizer: builds
# `make -C oracle sanitize` (the oracle library, the compiled drop-in caller, the local-BA host
# structure check), runs the host structure check, then the whole `pytest -m "not gpu"` suite with
# the sanitized oracle (ORB_ORACLE_LIB) and caller (ORB_SHIM_CALLER).  Python itself is not
# instrumented, so libasan / libubsan are preloaded; leak checking is off (the interpreter's
# own allocations at exit are not ours).  Runs in the build container (no GPU needed).
# usage: tools/sanitize_cpu.sh [extra pytest args]   (log: profiles/rNN_sanitize_cpu.txt by hand)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
make -s -C $R/oracle sanitize
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:alloc_dealloc_mismatch=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
$R/oracle/build/asan/lba_host_check
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 $R/oracle/build/asan/lba_host_check
export ORB_ORACLE_LIB=$R/oracle/build/asan/liborb_oracle.so
export ORB_SHIM_CALLER=$R/oracle/build/asan/shim_caller
LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)" \
    python -m pytest $R/tests -q -m "not gpu" -p no:cacheprovider "$@"
