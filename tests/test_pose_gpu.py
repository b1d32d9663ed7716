"""Optimizer::PoseOptimization on the GPU (batched, one workgroup per frame) against the CPU
oracle restatement: identical LM decisions (iterations per round, trials), identical outlier
flags and inlier counts, poses within 1e-5 (north_star tolerance)."""
import numpy as np
import pytest

import oracle_ref as O

pytestmark = pytest.mark.gpu


def _check(amd, frames, tol=1e-5):
    got = amd.PoseOptimization(frames)
    for f, g in zip(frames, got):
        ref = O.pose_optimization(f)
        assert g["iterations"] == ref["iterations"], (g["iterations"], ref["iterations"])
        assert g["trials"] == ref["trials"]
        assert g["n_inliers"] == ref["n_inliers"]
        assert np.array_equal(g["outlier"], ref["outlier"])
        assert np.abs(g["pose_q"] - ref["pose_q"]).max() < tol
        assert np.abs(g["pose_t"] - ref["pose_t"]).max() < tol


@pytest.mark.parametrize("kw", [
    dict(),                                            # monocular, 600 points, 10 % outliers
    dict(stereo_frac=0.5, seed=9),                     # mixed stereo / monocular
    dict(n_points=60, outlier_frac=0.3, seed=2),       # few points, many outliers
    dict(n_points=1500, seed=4, rot_noise=0.03, trans_noise=0.05),
    dict(stereo_frac=1.0, seed=14),                    # every edge stereo (EdgeStereoSE3ProjectXYZOnlyPose)
    dict(n_points=300, outlier_frac=0.6, seed=15),     # outliers the majority: many flips between rounds
    dict(n_points=1024, seed=16, rot_noise=0.05, trans_noise=0.1),   # the register path's largest frame, far start
    dict(n_points=11, seed=17),                        # just above the one-round limit (n >= 10: four rounds)
])
def test_pose_optimization_matches_oracle(amd, kw):
    from orb_slam2_amd import synth
    _check(amd, synth.pose_problems(n_frames=6, **kw))


def test_pose_optimization_edge_cases(amd):
    """Fewer than 3 correspondences: return 0, pose untouched; fewer than 10: one round only."""
    from orb_slam2_amd import synth
    frames = synth.pose_problems(n_frames=3, n_points=12, seed=8)
    frames[0] = {k: (v[:2] if k in ("obs", "xw", "info") else v) for k, v in frames[0].items()}
    frames[1] = {k: (v[:7] if k in ("obs", "xw", "info") else v) for k, v in frames[1].items()}
    got = amd.PoseOptimization(frames)
    q0, t0 = O.quat_from_Tcw(frames[0]["Tcw"])
    assert got[0]["n_inliers"] == 0 and np.array_equal(got[0]["pose_q"], q0) and np.array_equal(got[0]["pose_t"], t0)
    _check(amd, frames)


def test_pose_optimization_large_batch(amd):
    """A batch wider than the chip (one workgroup per frame) gives per-frame results independent
    of the batch composition."""
    from orb_slam2_amd import synth
    frames = synth.pose_problems(n_frames=300, n_points=200, seed=12, stereo_frac=0.2)
    all_ = amd.PoseOptimization(frames)
    part = amd.PoseOptimization(frames[100:103])
    for a, b in zip(all_[100:103], part):
        assert np.array_equal(a["pose_q"], b["pose_q"]) and np.array_equal(a["outlier"], b["outlier"])
    _check(amd, frames[::50])


def test_pose_optimization_vs_g2o_summation_order(amd):
    """The GPU against the oracle in g2o's own summation order (edges in order): the outcome
    (outlier flags, inlier count) identical and poses within 1e-5 (north_star); LM trial counts
    may differ where rho changes sign on a near-zero step (tests/test_pose_oracle_cpu.py), so
    they are reported, not asserted."""
    from orb_slam2_amd import synth
    frames = synth.pose_problems(n_frames=64, n_points=600, stereo_frac=0.3, seed=21)
    got = amd.PoseOptimization(frames)
    same = 0
    for f, g in zip(frames, got):
        ref = O.pose_optimization(f, g2o_order=True)
        assert np.array_equal(g["outlier"], ref["outlier"]) and g["n_inliers"] == ref["n_inliers"]
        assert np.abs(g["pose_q"] - ref["pose_q"]).max() < 1e-5
        assert np.abs(g["pose_t"] - ref["pose_t"]).max() < 1e-5
        same += g["trials"] == ref["trials"] and g["iterations"] == ref["iterations"]
    print(f"GPU vs g2o-order oracle: identical LM iterations and trials on {same}/{len(frames)} frames")
