"""Builds an instrumented variant of liborbslam2_amd.so with extra -D defines into
orb-slam2-_amd/lib/variant/ (select it with ORB_SLAM2_AMD_LIB=<path>).
Usage: python tools/build_variant.py NAME -DFOO=1 ..."""
import pathlib
import subprocess
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "orb-slam2-_amd"))
import build_lib  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
out = build_lib.LIB_DIR / "variant" / name
out.mkdir(parents=True, exist_ok=True)
objs = []
for s in build_lib.SOURCES:
    o = out / (pathlib.Path(s).stem + ".o")
    subprocess.check_call([build_lib.hipcc(), *build_lib.FLAGS, *defs, "-c", str(build_lib.CSRC / s), "-o", str(o)])
    objs.append(str(o))
lib = out / "liborbslam2_amd.so"
subprocess.check_call([build_lib.hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(lib), *objs])
print(lib)
