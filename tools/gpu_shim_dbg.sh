set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ORB_LBA_GROUP_DEBUG=1 timeout -k 10 200 python -u tools/grp_dbg.py > gpurun_out/gd1.log 2>&1 || true
grep -v amdgpu.ids gpurun_out/gd1.log | head -30
ORB_LBA_GROUP_HOST=1 ORB_LBA_GROUP_DEBUG=1 timeout -k 10 200 python -u tools/grp_dbg.py > gpurun_out/gd2.log 2>&1 || true
grep -v amdgpu.ids gpurun_out/gd2.log | head -30
