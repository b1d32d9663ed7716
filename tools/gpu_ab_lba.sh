# Same-box A/B of local-BA library variants (lib/variant/NAME, built by build_lba_variant.sh) and the
# working-tree build ("default"), interleaved over rounds: bench.py's config-4 and 60 / 200 KF corridor
# legs (extraction shortened, no CPU legs).  usage: gpu_ab_lba.sh "NAME1 NAME2 ..." [rounds]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in $(seq ${2:-2}); do
  for which in $1 default; do
    if [ $which = default ]; then unset ORB_SLAM2_AMD_LIB; else export ORB_SLAM2_AMD_LIB=$GRAFT_REPO_ROOT/orb-slam2-_amd/lib/variant/$which/liborbslam2_amd.so; fi
    timeout -k 10 300 python -u bench.py --no-cpu --no-stereo --no-extras --steps 3 --warmup 1 > gpurun_out/ab_lba.log 2>&1
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/ab_lba.log') if l.startswith('{')][-1])
s=d.get('lba_scaled', {}); l=d['lba']
print('$which', 'c4', l['ms_per_iter'], l['stage_ms_per_solve'], l['decisions']['trials'],
      *[(k, v.get('ms_per_iter'), v.get('trials_per_solve')) for k, v in s.items() if isinstance(v, dict)])"
  done
done
