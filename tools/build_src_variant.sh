# Builds a given extractor.hip (any path) as library variant NAME, the other objects from the current
# build, for same-box A/B runs (tools/gpu_ab_ext.sh NAME).  usage: build_src_variant.sh NAME FILE
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/pkg/csrc $T/include
cp $R/orb-slam2-_amd/csrc/* $T/pkg/csrc/ && cp $R/include/*.h $T/include/ && cp $2 $T/pkg/csrc/extractor.hip
V=$R/orb-slam2-_amd/lib/variant/$1
mkdir -p $V
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -c $T/pkg/csrc/extractor.hip -o $V/extractor.o
for f in matcher lba pose bow; do cp $R/orb-slam2-_amd/lib/$f.o $V/; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $V/liborbslam2_amd.so $V/*.o
rm -rf $T
echo $V/liborbslam2_amd.so
