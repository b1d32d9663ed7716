# quick reduced-solve harness run: n = 114 / 128 / 66, backward-solve mode $1 (default 0)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/ldlt2q.log
for a in "114 400 0" "114 400 1" "128 400 0" "66 200 0" "30 200 0"; do
  timeout -k 5 60 tools/micro/ldlt2 $a ${1:-0} >> gpurun_out/ldlt2q.log 2>&1
done
cat gpurun_out/ldlt2q.log
