# bit-identity of the local-BA outputs between variant base and the tree, then the LBA tests and timing
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ORB_SLAM2_AMD_LIB=$GRAFT_REPO_ROOT/orb-slam2-_amd/lib/variant/base/liborbslam2_amd.so timeout -k 5 120 python -u tools/lba_bits.py gpurun_out/bits_base.npz
timeout -k 5 120 python -u tools/lba_bits.py gpurun_out/bits_tree.npz
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/bits_base.npz"); b = np.load("gpurun_out/bits_tree.npz")
diff = [k for k in a.files if not np.array_equal(a[k], b[k])]
print("bit-identical" if not diff else f"differ: {diff}")
PY
bash tools/gpu_lba_round.sh ${1:-3}
