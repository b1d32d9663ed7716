"""Runs a few LocalBundleAdjustment solves of the config-4 problem and prints
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
    kw[k] = int(v)
pb = synth.ba_problem(**kw)
ba = amd.LocalBA()
for i in range(4):
    t0 = time.perf_counter()
    r = ba.solve(pb)
    dt = time.perf_counter() - t0
    print(f"solve {i}: {dt * 1e3:.3f} ms, iterations {r['iterations']}, trials {r['trials']}", flush=True)
