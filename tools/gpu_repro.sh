# bitwise reproducibility of local BA across solves, per library variant
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/repro.log
for v in nofuse cur; do
  echo "== $v" >> gpurun_out/repro.log
  if [ $v = cur ]; then L=orb-slam2-_amd/lib/liborbslam2_amd.so; else L=orb-slam2-_amd/lib/variant/$v/liborbslam2_amd.so; fi
  ORB_SLAM2_AMD_LIB=$L timeout -k 10 120 python -u tools/dbg_stop.py 2>&1 | head -1 >> gpurun_out/repro.log
done
