# The reduced-solve development harness (tools/micro/ldlt2.hip) on the GPU box: lane-primitive
# self-test, accuracy vs a CPU LDL^T and timing at several orders, both backward-solve modes.
# Output: gpurun_out/ldlt2.log
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/ldlt2.log
for m in 0 1; do
for a in "114 400 0" "114 400 1" "128 400 0" "120 200 0" "66 200 0" "30 200 0" "6 200 0" "96 200 0"; do
  timeout -k 5 60 tools/micro/ldlt2 $a $m >> gpurun_out/ldlt2.log 2>&1
done
done
cat gpurun_out/ldlt2.log
