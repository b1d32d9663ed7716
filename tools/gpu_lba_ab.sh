# LBA solve time A/B over an environment setting: tools/gpu_lba_ab.sh VAR "A B C" (interleaved, 3 rounds)
set -e
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for i in 1 2 3; do
  for v in $2; do
    echo -n "$1=$v " >> gpurun_out/lba_ab.log
    env $1=$v timeout -k 10 120 python -u tools/lba_timing.py 2>&1 | tail -1 >> gpurun_out/lba_ab.log
  done
done
echo ok
