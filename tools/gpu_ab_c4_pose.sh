# Same-box A/B of a library variant (lib/variant/NAME) against the working-tree build on the config-4
# local BA (tools/lba_timing.py median) and one-frame PoseOptimization (tools/pose_timing.py),
# interleaved over rounds.  usage: gpu_ab_c4_pose.sh NAME [rounds]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in $(seq ${2:-2}); do
  for which in $1 default; do
    if [ $which = default ]; then unset ORB_SLAM2_AMD_LIB; else export ORB_SLAM2_AMD_LIB=$GRAFT_REPO_ROOT/orb-slam2-_amd/lib/variant/$which/liborbslam2_amd.so; fi
    a=$(timeout -k 10 120 python -u tools/lba_timing.py solves=16 | grep median)
    b=$(timeout -k 10 120 python -u tools/pose_timing.py 40 | tail -1)
    echo "$which | c4 $a | pose $b"
  done
done
