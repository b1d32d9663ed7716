"""Writes the config-4 local-BA window (synth.ba_problem, 20 KF x 3000 points) in shim_caller's lba input
format (the arrays bench.py's routed LocalBundleAdjustment row writes).  usage: mk_lba_in.py OUT"""
import sys, numpy as np, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pkgload; amd=pkgload.load()
from orb_slam2_amd import synth
pb = synth.ba_problem(n_local=20, n_points=3000)
inv_sigma2 = (np.float32(1.0) / np.array([np.float32(1.2) ** (2 * lv) for lv in range(8)], np.float32))
octave = np.array([int(np.argmin(np.abs(inv_sigma2.astype(np.float64) - i))) for i in pb["edge_info"]], np.int32)
arrays = [np.asarray(pb["Tcw"], np.float32).reshape(-1), np.asarray(pb["pose_fixed"], np.uint8),
          np.asarray(pb["pose_id"], np.int64), np.asarray(pb["point_xyz"], np.float32).reshape(-1),
          np.asarray(pb["point_id"], np.int64), np.asarray(pb["edge_point"], np.int32),
          np.asarray(pb["edge_pose"], np.int32), np.asarray(pb["edge_obs"], np.float32).reshape(-1), octave,
          np.asarray(pb["edge_cam"][0], np.float32), inv_sigma2, np.zeros(1, np.uint8)]
with open(sys.argv[1], "wb") as f:
    for a in arrays:
        a = np.ascontiguousarray(a)
        np.array([a.size], np.int64).tofile(f)
        a.tofile(f)
