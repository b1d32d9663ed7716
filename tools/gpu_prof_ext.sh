# rocprofv3 kernel trace of the extraction + matching step only (config 2 bench) -> gpurun_out/prof_ext
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_ext -o ext -- \
    python3 $R/bench.py --no-cpu --no-lba --no-extras --no-stereo --steps 20 --warmup 5 "$@" > $R/gpurun_out/prof_ext.log 2>&1
cd $R
python3 tools/trace_by_shape.py gpurun_out/prof_ext/ext_kernel_trace.csv > gpurun_out/prof_ext.txt
