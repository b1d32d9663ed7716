"""Solves config 4, a mixed stereo window, a small window and a 60 KF corridor (the multi-workgroup
reduced solve) through the loaded library and saves every output array (A/B bit-identity checks
between library variants: ORB_SLAM2_AMD_LIB selects one).
python tools/lba_bits.py OUT.npz"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import pkgload  # noqa: E402

amd = pkgload.load()
from orb_slam2_amd import synth  # noqa: E402

out = {}
for tag, kw in (("c4", dict()), ("st", dict(stereo_frac=0.5, seed=7)), ("small", dict(n_local=9, n_fixed=2, n_points=900, seed=5))):
    r = amd.LocalBA().solve(synth.ba_problem(**kw))
    for k in ("pose_q", "pose_t", "point_xyz", "trace", "edge_erase", "edge_chi2"):
        out[f"{tag}_{k}"] = np.asarray(r[k])
for tag, kw in (("kf60", dict(n_local=60, n_fixed=4, n_points=8000, seed=21)),):
    r = amd.LocalBA().solve(synth.ba_problem_corridor(**kw))
    for k in ("pose_q", "pose_t", "point_xyz", "trace", "edge_erase", "edge_chi2"):
        out[f"{tag}_{k}"] = np.asarray(r[k])
np.savez(sys.argv[1], **out)
print("saved", len(out))
