"""Where the GPU SearchByProjection(Frame, KF) and the oracle part on the wide-window case."""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import pkgload  # noqa: E402

amd = pkgload.load()
import test_sbp_kf as T  # noqa: E402

for seed, th, od in ((7, 40.0, 200), (7, 10.0, 100), (3, 40.0, 200)):
    for ori in (False, True):
        p, kf, kfs, occ = T._problem(seed)
        rn, rm = T._oracle(p, kf, kfs, occ, th, od, ori)
        kp = p["kp"]
        m = amd.ORBmatcher(0.75, ori)
        n, gm = m.SearchByProjectionKF(T._frame(kf, kp), T._frame(kfs, None), p["mp_valid"], p["mp_xyz"],
                                       p["mp_min_dist"], p["mp_max_dist"], p["mp_desc"], kp["cam"][:4], kp["Ow"],
                                       kp["log_scale_factor"], th, od, occ)
        m.close()
        diff = np.flatnonzero(gm != rm)
        print(f"seed {seed} th {th} od {od} ori {ori}: gpu {n} oracle {rn} differing slots {len(diff)}", flush=True)
        for s in diff[:8]:
            print(f"   slot {s}: gpu {gm[s]} oracle {rm[s]} angle {kf['angle'][s]:.3f}", flush=True)
