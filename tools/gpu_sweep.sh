set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/sweep.log
for a in "--streams 3 --batch 384" "--streams 2 --batch 512" "--streams 4 --batch 512" "--streams 3 --batch 576" "--streams 2 --batch 384" "--streams 3 --batch 384" "--streams 2 --batch 512"; do
  echo "== $a" >> gpurun_out/sweep.log
  timeout -k 10 120 python -u bench.py --no-cpu --no-lba --no-extras --no-stereo --steps 20 $a 2>&1 | tail -1 | cut -c1-120 >> gpurun_out/sweep.log
done
echo ok
