# Same-box A/B of several extraction library variants (lib/variant/NAME, built by build_head_variant.sh /
# build_src_variant.sh) and the working-tree build ("default"), interleaved over rounds, bench.py's default
# extraction step without the CPU / LBA / stereo legs.  usage: gpu_ab_multi.sh "NAME1 NAME2 ..." [rounds]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in $(seq ${2:-2}); do
  for which in $1 default; do
    if [ $which = default ]; then unset ORB_SLAM2_AMD_LIB; else export ORB_SLAM2_AMD_LIB=$GRAFT_REPO_ROOT/orb-slam2-_amd/lib/variant/$which/liborbslam2_amd.so; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-lba --no-stereo --no-extras ${AB_ARGS:---no-profile} --steps ${AB_STEPS:-30} --warmup 5 > gpurun_out/ab.log 2>&1
    python -c "import json; d=json.loads([l for l in open('gpurun_out/ab.log') if l.startswith('{')][-1]); print('$which', d['value'], d['ms_per_step'])"
  done
done
