# Same-box A/B of the extraction step: k_pyramid LDS budgets (ORB_PYR_LDS_KB, with level 0 read in
# place) and the round-3 behaviour of copying level 0 into the slab (ORB_L0_COPY=1), alternating,
# two rounds.  Usage: gpurun -- bash tools/gpu_sweep_l0.sh  (PYR_KBS="24 32 40 52" by default)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
one() {   # $1 label, env in the caller
  timeout -k 10 200 python -u bench.py --no-cpu --no-lba --no-stereo --no-extras --no-profile --steps 30 --warmup 5 > gpurun_out/sweep.log 2>&1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/sweep.log') if l.startswith('{')][-1]); print('$1', d['value'], d['ms_per_step'])"
}
for round in 1 2; do
  for pk in ${PYR_KBS:-24 32 40 52}; do
    ORB_PYR_LDS_KB=$pk one "round $round pyr_kb $pk in-place"
  done
  ORB_PYR_LDS_KB=52 ORB_L0_COPY=1 one "round $round pyr_kb 52 l0-copy"
done
