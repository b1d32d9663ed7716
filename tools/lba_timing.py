"""Runs a few LocalBundleAdjustment solves of the config-4 problem (corridor=1 n_local=200
n_points=100000: the scaled window) and prints
per-stage event times; with ORB_SLAM2_AMD_LIB pointing at an ORB_TIMING variant
(tools/build_variant.py timing -DORB_TIMING) the kernels print their own clock splits."""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import pkgload  # noqa: E402

amd = pkgload.load()
from orb_slam2_amd import synth  # noqa: E402

kw = {}
for a in sys.argv[1:]:
    k, v = a.split("=")
    kw[k] = float(v) if "." in v else int(v)
# corridor=1: the scaled window generator (synth.ba_problem_corridor, banded covisibility)
gen = synth.ba_problem_corridor if kw.pop("corridor", 0) else synth.ba_problem
pb = gen(**kw)
print(f"problem: {len(pb['Tcw'])} keyframes, {len(pb['point_xyz'])} points, {len(pb['edge_point'])} edges", flush=True)
ba = amd.LocalBA()
n = 12
call = ba.prepared(pb)
ts = []
for i in range(n):
    t0 = time.perf_counter()
    its, trials, _ = call()
    dt = time.perf_counter() - t0
    ts.append(dt)
    print(f"solve {i}: {dt * 1e3:.3f} ms, iterations {its}, trials {trials}", flush=True)
import statistics  # noqa: E402
print(f"median of solves 4..{n - 1}: {1e3 * statistics.median(ts[4:]):.3f} ms", flush=True)
