"""lba_group debugging aid: repeated group solves of one synthetic window, reporting per-rank
flag words (ORB_LBA_GROUP_DEBUG=1) and agreement with a single context."""
import sys
import numpy as np
sys.path.insert(0, ".")
import pkgload
amd = pkgload.load()
from orb_slam2_amd import synth
kw = dict(n_local=8, n_fixed=3, n_points=900, stereo_frac=0.4, seed=11)
for a in sys.argv[1:]:
    k, v = a.split("=")
    kw[k] = float(v) if "." in v else int(v)
pb = synth.ba_problem(**kw)
one = amd.LocalBA().solve(pb)
print("single", one["iterations"], one["trials"], flush=True)
for i in range(4):
    grp = amd.LocalBAGroup([0, 0])
    try:
        r = grp.solve(pb)
        print("group", i, r["iterations"], r["trials"], "same" if r["iterations"] == one["iterations"] else "DIFF", flush=True)
    except Exception as e:
        print("group", i, "failed", e, flush=True)
    grp.close()
