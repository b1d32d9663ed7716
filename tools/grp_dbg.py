import sys, os
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import pkgload
amd = pkgload.load()
from orb_slam2_amd import synth
pb = synth.ba_problem()
grp = amd.LocalBAGroup([0, 0])
for i in range(3):
    try:
        r = grp.solve(pb)
        print("solve", i, "ok", r["iterations"], r["trials"], flush=True)
    except Exception as e:
        print("solve", i, "failed", e, flush=True)
