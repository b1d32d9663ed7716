set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/dbg_repro.py > gpurun_out/dbg_repro.log 2>&1
bash tools/gpu_ldlt.sh
