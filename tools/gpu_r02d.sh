set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for a in "" "--no-match-stream" "--streams 3 --batch 192" "--streams 2 --batch 256" "--streams 1 --batch 64"; do
  echo "== $a" >> gpurun_out/sweep.log
  timeout -k 10 120 python -u bench.py --no-cpu --no-lba --no-extras --no-stereo $a 2>&1 | tail -1 | cut -c1-200 >> gpurun_out/sweep.log
done
echo ok
