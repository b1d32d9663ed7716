"""ORBmatcher::SearchBySim3 (R/src/ORBmatcher.cpp:1305-1503, LoopClosing::ComputeSim3): the oracle
pairs the keypoints of the same 3-D point (CPU); both gfx950 projection directions + the host
mutual check bit-exact against the oracle for three Sim3 scales and two radii (GPU)."""
import numpy as np
import pytest

import oracle_ref as O


def _problem(seed=6, s12=1.0):
    from orb_slam2_amd import synth
    return synth.sim3_problem(seed=seed, s12=s12)


def test_oracle_pairs_same_points():
    p = _problem()
    n, m = O.search_by_sim3(p, 7.5)
    k1, k2 = p["kf1"], p["kf2"]
    i1 = np.flatnonzero(m >= 0)
    assert n == len(i1) and n > 100
    same = k1["point"][i1] == k2["point"][m[i1]]
    assert same.mean() > 0.95


def _frame(k):
    from orb_slam2_amd import Frame
    a = np.zeros(len(k["x"]), dtype=[("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
    a["x"], a["y"], a["octave"] = k["x"], k["y"], k["octave"]
    return Frame(a, k["desc"], k["W"], k["H"])


@pytest.mark.gpu
@pytest.mark.parametrize("seed,s12,th", [(6, 1.0, 7.5), (8, 1.03, 7.5), (9, 0.97, 4.0)])
def test_search_by_sim3_gpu(amd, seed, s12, th):
    from orb_slam2_amd import synth
    p = _problem(seed, s12)
    rn, rm = O.search_by_sim3(p, th)
    S1, S2 = synth.sim3_side_transforms(p)
    sides = []
    for k, S in ((p["kf1"], S1), (p["kf2"], S2)):
        sides.append(dict(Tcw=k["Tcw"], S=S, valid=k["mp_valid"], xyz=k["mp_xyz"], min_dist=k["mp_min_dist"],
                          max_dist=k["mp_max_dist"], desc=k["mp_desc"]))
    sc = (p["log_scale_factor"], p["scale_factors"])
    n, m = amd.SearchBySim3(_frame(p["kf1"]), _frame(p["kf2"]), sides[0], sides[1], p["cam"], sc, sc, th)
    assert n == rn and np.array_equal(m, rm) and n > 0
