# same-box A/B of the local-BA solve: variant/base (a git revision) vs the working tree, alternated
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/ab_lba.log
for i in 1 2 3; do
  ORB_SLAM2_AMD_LIB=orb-slam2-_amd/lib/variant/base/liborbslam2_amd.so timeout -k 10 120 python -u tools/lba_timing.py | tail -1 | sed 's/^/base: /' >> gpurun_out/ab_lba.log
  timeout -k 10 120 python -u tools/lba_timing.py | tail -1 | sed 's/^/new:  /' >> gpurun_out/ab_lba.log
done
