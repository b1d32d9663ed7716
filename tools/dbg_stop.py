import sys, pathlib
sys.path[:0] = ['/root/repo', '/root/repo/tests']
import pkgload
amd = pkgload.load()
import numpy as np
from orb_slam2_amd import optimizer, synth
import test_lba_gpu as T
pb = T._problem(amd, n_local=12, n_fixed=2, n_points=1200, seed=31, outlier_frac=0.2)
full = amd.LocalBA().solve(pb, optimizer.options(5, 40, fixed_iterations=True))
full2 = amd.LocalBA().solve(pb, optimizer.options(5, 40, fixed_iterations=True))
print("full iters", full["iterations"], full["trials"], "repro", np.array_equal(full["trace"], full2["trace"]))
qmax = full["trace"][:, 3].astype(int)
print("qmax", qmax.tolist())
ks = [k for k in range(5, len(qmax)) if qmax[k] >= 2]
k = ks[0]; before = int(qmax[:k].sum())
print("k", k, "before", before)
for extra in (0, 1):
    ctx = amd.LocalBA(); ctx.debug_stop_after_trials(before + 1 + extra)
    got = ctx.solve(pb, optimizer.options(5, 40, fixed_iterations=True))
    print("stop", before + 1 + extra, "iters", got["iterations"], "trials", got["trials"], "qmax", got["trace"][:, 3].astype(int).tolist())
