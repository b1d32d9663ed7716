"""Matcher handle lifetime check: create / use / drop without close() / collect, per call form, each
case in its own process (an abort in one does not hide the others)."""
import subprocess
import sys

CASE = r'''
import gc, sys, pathlib
import numpy as np
ROOT = pathlib.Path(sys.argv[1]); sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import pkgload; amd = pkgload.load()
from orb_slam2_amd import synth
import test_sbp_kf as T
mode = sys.argv[2]
p, kf, kfs, occ = T._problem(3)
kp = p["kp"]
for rep in range(3):
    m = amd.ORBmatcher(0.75, True)
    if mode in ("sbpkf", "sbpkf_close"):
        n, gm = m.SearchByProjectionKF(T._frame(kf, kp), T._frame(kfs, None), p["mp_valid"], p["mp_xyz"], p["mp_min_dist"],
                                       p["mp_max_dist"], p["mp_desc"], kp["cam"][:4], kp["Ow"], kp["log_scale_factor"],
                                       10.0, 100, occ)
    if mode.endswith("close"):
        m.close()
    del m
    gc.collect()
    print(mode, "rep", rep, "ok", flush=True)
'''
for mode in ("none", "none_close", "sbpkf", "sbpkf_close"):
    r = subprocess.run([sys.executable, "-c", CASE, sys.argv[1], mode], capture_output=True, text=True, timeout=120)
    print(mode, "rc", r.returncode, r.stdout.strip().replace("\n", " | "), r.stderr.strip()[-300:], flush=True)
