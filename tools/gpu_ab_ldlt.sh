# Local-BA A/B of the reduced solve: ORB_LBA_LDLT_OLD=1 (k_ldlt_solve<true>) against the default
# (k_ldlt_df), interleaved, bench.py's config-4 / 60 KF / 200 KF legs; then the LBA / global-BA tests.
# usage: gpu_ab_ldlt.sh [rounds]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lba_gpu.py tests/test_global_ba.py tests/test_lba_dist_gpu.py tests/test_lba_group_gpu.py tests/test_cpp_shim.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lbatest.log 2>&1 || { tail -40 gpurun_out/lbatest.log; exit 1; }
tail -2 gpurun_out/lbatest.log
for i in $(seq ${1:-2}); do
  for which in old df; do
    if [ $which = old ]; then export ORB_LBA_LDLT_OLD=1; else unset ORB_LBA_LDLT_OLD; fi
    timeout -k 10 300 python -u bench.py --no-cpu --no-stereo --no-extras --steps 3 --warmup 1 > gpurun_out/ab_lba.log 2>&1
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/ab_lba.log') if l.startswith('{')][-1])
s=d.get('lba_scaled', {}); l=d['lba']
print('$which', 'c4', l['ms_per_iter'], l['stage_ms_per_solve'], l['decisions']['trials'],
      *[(k, v.get('ms_per_iter'), v.get('trials_per_solve')) for k, v in s.items() if isinstance(v, dict)])"
  done
done
