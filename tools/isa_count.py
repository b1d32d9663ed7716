"""Static instruction mix per kernel of one HIP source (gfx950 device asm): counts of VALU (v_*),
SALU (s_*), LDS (ds_*), vector memory (buffer_/global_/flat_) and MFMA instructions in each
kernel's body.  Static counts, not executed ones: use it to compare two versions of a kernel's
inner loop before spending a GPU run.  usage: python tools/isa_count.py [SRC] [KERNEL_SUBSTR ...]
"""
import pathlib
import re
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam2-_amd"))
import build_lib  # noqa: E402


def kernel_mix(src, want=()):
    asm = subprocess.run([build_lib.hipcc(), *build_lib.FLAGS, "-I", str(ROOT / "include"), "--cuda-device-only", "-S",
                          "-o", "-", str(src)], capture_output=True, text=True, check=True).stdout
    out, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", line)
        if m and not m.group(1).startswith(".") and not m.group(1).startswith("$"):
            name = m.group(1)
            cur = name if (not want or any(w in name for w in want)) else None
            if cur:
                out.setdefault(cur, {"valu": 0, "salu": 0, "lds": 0, "vmem": 0, "mfma": 0, "total": 0})
            continue
        if cur is None:
            continue
        t = line.strip()
        if t.startswith(".end_amdhsa_kernel") or t.startswith(".Lfunc_end"):
            cur = None
            continue
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        c = out[cur]
        c["total"] += 1
        if "mfma" in op:
            c["mfma"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("buffer_", "global_", "flat_")):
            c["vmem"] += 1
    return out


if __name__ == "__main__":
    src = pathlib.Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "orb-slam2-_amd/csrc/extractor.hip"
    for k, v in kernel_mix(src, sys.argv[2:]).items():
        print(f"{k[:60]:60s} " + " ".join(f"{a}={b}" for a, b in v.items()))
