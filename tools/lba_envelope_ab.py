"""Same-process A/B of the multi-workgroup reduced solve's variants on the 60 KF and 200 KF corridor
windows, interleaved: "split" = the dense passes with two launches per panel (ORB_LBA_MW_DENSE=1
ORB_LBA_MW_SPLIT=1, the round-5 form), "envelope" = the envelope skipping with two launches per
panel (ORB_LBA_MW_SPLIT=1), "fused" = the default (envelope + k_ldlt_mw_step).  The results are
compared bitwise (skipped work adds exact zeros and the fused panel forms the same tiles, so the
estimates, the edge chi2 and the LM decisions must be identical).
usage: python tools/lba_envelope_ab.py [rounds] [solves per round]"""
import os
import pathlib
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import pkgload  # noqa: E402

amd = pkgload.load()
from orb_slam2_amd import synth  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
per = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ok = True
for nl, npts in ((60, 8000), (200, 100000)):
    pb = synth.ba_problem_corridor(n_local=nl, n_fixed=4, n_points=npts)
    ba = amd.LocalBA()
    call = ba.prepared(pb)
    modes = {"split": {"ORB_LBA_MW_DENSE": "1", "ORB_LBA_MW_SPLIT": "1"}, "envelope": {"ORB_LBA_MW_SPLIT": "1"},
             "fused": {}}
    ms = {k: [] for k in modes}
    res = {}
    for r in range(rounds):
        for mode, env in modes.items():
            for k in ("ORB_LBA_MW_DENSE", "ORB_LBA_MW_SPLIT"):
                os.environ.pop(k, None)
            os.environ.update(env)
            call()   # warm (graphs of this mode)
            for _ in range(per):
                t0 = time.perf_counter()
                its, trials, keep = call()
                dt = time.perf_counter() - t0
                ms[mode].append(1e3 * dt / max(1, sum(its)))
            out = keep[3]
            snap = (its, trials, out["pose_q"].copy(), out["pose_t"].copy(), out["point_xyz"].copy(),
                    out["edge_chi2"].copy())
            if mode in res:
                continue
            res[mode] = snap
    for k in ("ORB_LBA_MW_DENSE", "ORB_LBA_MW_SPLIT"):
        os.environ.pop(k, None)
    a = res["split"]
    line = [f"{nl} KF x {npts}: ms/iter"]
    for mode in modes:
        line.append(f"{mode} {statistics.median(ms[mode]):.4f} (min {min(ms[mode]):.4f})")
    line.append(f"iterations {a[0]} trials {a[1]}")
    for mode in ("envelope", "fused"):
        b = res[mode]
        same = a[0] == b[0] and a[1] == b[1] and all(np.array_equal(x, y) for x, y in zip(a[2:], b[2:]))
        ok &= same
        line.append(f"{mode} bitwise = split: {same}")
        if not same:
            for name, x, y in zip(("q", "t", "X", "chi2"), a[2:], b[2:]):
                line.append(f"{mode} {name} max|diff| {np.max(np.abs(x - y)):.3e}")
    print("; ".join(line), flush=True)
sys.exit(0 if ok else 1)
