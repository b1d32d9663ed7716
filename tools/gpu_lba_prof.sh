# LBA: ORB_TIMING clock split + a rocprofv3 kernel trace of tools/lba_timing.py
set -e
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ORB_SLAM2_AMD_LIB=$R/orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so timeout -k 10 120 python -u tools/lba_timing.py > gpurun_out/lba_timing.log 2>&1
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_lba -o lba -- python3 $R/tools/lba_timing.py > $R/gpurun_out/prof_lba.log 2>&1
cd $R && python tools/lba_trace.py $(ls gpurun_out/prof_lba/*/lba_kernel_trace.csv gpurun_out/prof_lba/lba_kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/lba_trace.txt 2>&1
echo ok
