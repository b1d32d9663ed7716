# memory-hierarchy PMC passes over the 200 KF corridor solve (kernels one by one): L2 -> HBM/MALL
# fetch, L1 -> L2 read requests, L2 hits; per kernel per launch -> gpurun_out/lba_mem_kf200.txt
set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp ORB_LBA_NO_GRAPH=1
cd /tmp
ARGS="corridor=1 n_local=200 n_points=100000 solves=2"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/lmem_a -o run -- python3 $R/tools/lba_timing.py $ARGS > $R/gpurun_out/lmem_a.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/lmem_b -o run -- python3 $R/tools/lba_timing.py $ARGS > $R/gpurun_out/lmem_b.log 2>&1
cd $R && python - <<'PY' > gpurun_out/lba_mem_kf200.txt
import sys
sys.path.insert(0, "tools")
from pmc_traffic import per_kernel
a = per_kernel("gpurun_out/lmem_a"); b = per_kernel("gpurun_out/lmem_b")
for k in sorted(a, key=lambda k: -a[k].get("FETCH_SIZE", 0)):
    if k not in b: continue
    print(f"{k:28s} fetch(x2) {2*a[k].get('FETCH_SIZE',0)/1024:9.2f} MB  write {b[k].get('WRITE_SIZE',0)/1024:8.2f} MB  "
          f"TCC_HIT {a[k].get('TCC_HIT_sum',0)/1e6:8.3f} M  TCP->TCC rd {b[k].get('TCP_TCC_READ_REQ_sum',0)/1e6:8.3f} M  "
          f"TCP acc {b[k].get('TCP_TOTAL_CACHE_ACCESSES_sum',0)/1e6:8.3f} M  n={a[k]['dispatches']}")
PY
cat gpurun_out/lba_mem_kf200.txt | head -12
