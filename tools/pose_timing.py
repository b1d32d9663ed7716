"""One-frame PoseOptimization through the C-ABI, as bench.py's single-call row (600 points, 30 %
stereo); with the ORB_TIMING library variant the kernel prints its per-phase cycle split.
python tools/pose_timing.py [reps]"""
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import pkgload  # noqa: E402

amd = pkgload.load()
from orb_slam2_amd import synth  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
fr = synth.pose_problems(n_frames=1, n_points=600, stereo_frac=0.3, seed=21)
ts = []
for _ in range(reps):
    t0 = time.perf_counter()
    amd.PoseOptimization(fr)
    ts.append(time.perf_counter() - t0)
print("one-frame PoseOptimization (Python binding) median us:", round(1e6 * float(np.median(ts)), 1), flush=True)
