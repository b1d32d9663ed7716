set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ORB_LBA_GROUP_DEBUG=1 timeout -k 10 60 python -u tools/grp_dbg.py > gpurun_out/grp_dbg.log 2>&1; cat gpurun_out/grp_dbg.log | grep -v amdgpu.ids
ORB_LBA_NO_GRAPH=1 ORB_LBA_GROUP_DEBUG=1 timeout -k 10 60 python -u tools/grp_dbg.py > gpurun_out/grp_dbg2.log 2>&1; cat gpurun_out/grp_dbg2.log | grep -v amdgpu.ids
