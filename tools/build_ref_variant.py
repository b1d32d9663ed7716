"""Builds liborbslam2_amd.so from the sources of a git revision (default HEAD) into
orb-slam2-_amd/lib/variant/<name>/, for same-box A/B timing against the working tree.
usage: python tools/build_ref_variant.py NAME [REV]"""
import pathlib
import subprocess
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam2-_amd"))
import build_lib  # noqa: E402

name = sys.argv[1]
rev = sys.argv[2] if len(sys.argv) > 2 else "HEAD"
out = build_lib.LIB_DIR / "variant" / name
out.mkdir(parents=True, exist_ok=True)
with tempfile.TemporaryDirectory() as td:
    src = pathlib.Path(td) / "orb-slam2-_amd" / "csrc"
    src.mkdir(parents=True)
    (pathlib.Path(td) / "include").mkdir()
    files = subprocess.check_output(["git", "ls-tree", "--name-only", rev, "orb-slam2-_amd/csrc/", "include/"],
                                    cwd=ROOT, text=True).split()
    for f in files:
        data = subprocess.check_output(["git", "show", f"{rev}:{f}"], cwd=ROOT)
        (pathlib.Path(td) / f).write_bytes(data)
    objs = []
    for s in build_lib.SOURCES:
        o = out / (pathlib.Path(s).stem + ".o")
        subprocess.check_call([build_lib.hipcc(), *build_lib.FLAGS, "-c", str(src / s), "-o", str(o)])
        objs.append(str(o))
    lib = out / "liborbslam2_amd.so"
    subprocess.check_call([build_lib.hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(lib), *objs])
print(lib)
