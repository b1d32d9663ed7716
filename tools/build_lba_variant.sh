# Builds a given lba.hip (any path) as library variant NAME, the other objects from the current build,
# for same-box A/B runs of the local-BA legs (tools/gpu_ab_lba.sh).  usage: build_lba_variant.sh NAME FILE
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/pkg/csrc $T/include
cp $R/orb-slam2-_amd/csrc/* $T/pkg/csrc/ && cp $R/include/*.h $T/include/ && cp $2 $T/pkg/csrc/lba.hip
V=$R/orb-slam2-_amd/lib/variant/$1
mkdir -p $V
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -c $T/pkg/csrc/lba.hip -o $V/lba.o
for f in extractor matcher pose bow; do cp $R/orb-slam2-_amd/lib/$f.o $V/; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $V/liborbslam2_amd.so $V/*.o
rm -rf $T
echo $V/liborbslam2_amd.so
