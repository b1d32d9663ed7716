# Diagnostic sweep of the extraction step: LDS budgets ORB_OT_LDS_KB (k_octree, 0 = the library's
# default) / ORB_PYR_LDS_KB (k_pyramid) and streams:frames-per-step pairs.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for pk in ${PYR_KBS:-52}; do
for kb in ${OT_KBS:-0}; do
  for st in ${STREAMS:-"3:384" "4:512"}; do
  s=${st%%:*}; b=${st##*:}
  ORB_PYR_LDS_KB=$pk ORB_OT_LDS_KB=$kb timeout -k 10 200 python -u bench.py --no-cpu --no-lba --no-stereo --no-extras --no-profile --streams $s --batch $b --steps 30 --warmup 5 > gpurun_out/sweep.log 2>&1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/sweep.log') if l.startswith('{')][-1]); print('pyr_kb $pk ot_kb $kb streams $s batch $b', d['value'], d['ms_per_step'])"
  done
done
done
