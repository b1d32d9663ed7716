"""Builds liborbslam2_amd.so (hand-written HIP for gfx950) in-tree with hipcc.

The shared library is the product: a C-ABI (include/orbslam2_amd.h) over the
kernels in csrc/.  -ffp-contract=off pins FP contraction off on host and
device so every float result matches the oracle bit for bit.
"""
import os
import pathlib
import shutil
import subprocess
import sys

PKG = pathlib.Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIB_DIR = PKG / "lib"
LIB = LIB_DIR / "liborbslam2_amd.so"
SOURCES = ["extractor.hip", "matcher.hip", "lba.hip", "pose.hip", "bow.hip"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-Wall", "-Wno-unused-function", "-Wno-unused-result"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and pathlib.Path(c).exists():
            return c
    raise RuntimeError("hipcc not found: the HIP library cannot be built")


def build(force: bool = False, verbose: bool = False) -> pathlib.Path:
    srcs = [CSRC / s for s in SOURCES if (CSRC / s).exists()]
    deps = srcs + list(CSRC.glob("*.h")) + list(CSRC.glob("*.inc")) + [PKG.parent / "include" / "orbslam2_amd.h"]
    if LIB.exists() and not force and all(LIB.stat().st_mtime >= d.stat().st_mtime for d in deps):
        return LIB
    LIB_DIR.mkdir(exist_ok=True)
    objs = []
    for s in srcs:
        o = LIB_DIR / (s.stem + ".o")
        cmd = [hipcc(), *FLAGS, "-c", str(s), "-o", str(o)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        objs.append(str(o))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(tmp), *objs]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    check_isa(srcs, verbose)
    return LIB


# ROCm 7.2 lowers a clamp-of-ashr pair to v_ashr_pk_u8_i32 without clearing the
# destination's high half, which then leaks into a packed word (seen in k_blur).
# Every kernel source is checked for that instruction after the build.
BANNED = ("v_ashr_pk_u8_i32", "v_ashr_pk_i8_i32")


def check_isa(srcs, verbose=False):
    for s in srcs:
        asm = subprocess.run([hipcc(), *FLAGS, "--cuda-device-only", "-S", "-o", "-", str(s)],
                             check=True, capture_output=True, text=True).stdout
        bad = [b for b in BANNED if b in asm]
        if bad:
            raise RuntimeError(f"{s.name}: banned instruction(s) {bad} in device code")
        if verbose:
            print(f"isa check ok: {s.name}", flush=True)


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
