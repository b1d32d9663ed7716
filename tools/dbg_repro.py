import sys
sys.path[:0] = ['/root/repo', '/root/repo/tests']
import pkgload
amd = pkgload.load()
import numpy as np
from orb_slam2_amd import optimizer
import test_lba_gpu as T
pb = T._problem(amd, n_local=12, n_fixed=2, n_points=1200, seed=31, outlier_frac=0.2)
runs = [amd.LocalBA().solve(pb, optimizer.options(5, 40, fixed_iterations=True)) for _ in range(4)]
ctx = amd.LocalBA()
runs += [ctx.solve(pb, optimizer.options(5, 40, fixed_iterations=True)) for _ in range(3)]
base = runs[0]["trace"]
for i, r in enumerate(runs[1:], 1):
    tr = r["trace"]
    n = min(len(tr), len(base))
    diff = [k for k in range(n) if not np.array_equal(tr[k], base[k])]
    print(i, "rows", len(tr), len(base), "first diff row", diff[:1], "pose equal", np.array_equal(r["pose_q"], runs[0]["pose_q"]))
    if diff:
        k = diff[0]
        print("   base", base[k].tolist(), " run", tr[k].tolist())
