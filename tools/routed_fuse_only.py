"""Times only the Fuse / SearchForTriangulation / SearchByBoW routed calls (bench.py's synthetic
inputs) for tracing the per-call floor: python tools/routed_fuse_only.py [reps]"""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import pkgload  # noqa: E402

amd = pkgload.load()
from orb_slam2_amd import synth, Frame  # noqa: E402

torch.cuda.init()
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
fp = synth.fuse_problem()
kf, kp = fp["kf"], fp["kp"]
a = np.zeros(len(kf["x"]), dtype=[("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                                  ("octave", "<i4"), ("class_id", "<i4")])
a["x"], a["y"], a["octave"] = kf["x"], kf["y"], kf["octave"]
ff = Frame(a, kf["desc"], kf["W"], kf["H"], mvuRight=kf["uright"])
fargs = (fp["mp_valid"], fp["mp_xyz"], fp["mp_normal"], fp["mp_min_dist"], fp["mp_max_dist"], fp["mp_desc"])


def fuse():
    return amd.Fuse(ff, kp["Tcw"], kp["Ow"], kp["cam"], kp["log_scale_factor"], kp["scale_factors"],
                    kp["inv_level_sigma2"], *fargs, 3.0)


for _ in range(20):
    fuse()
ts = []
for _ in range(reps):
    t0 = time.perf_counter()
    fuse()
    ts.append(time.perf_counter() - t0)
print("fuse median us", round(1e6 * float(np.median(ts)), 1), "min", round(1e6 * min(ts), 1))
