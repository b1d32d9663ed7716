"""ORBmatcher::SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th) (R/src/ORBmatcher.cpp:
370-497, LoopClosing::ComputeSim3): the oracle finds the planted points (CPU); the gfx950
candidate kernel + sequential replay bit-exact against the oracle with pre-set vpMatched slots
(GPU)."""
import numpy as np
import pytest

import oracle_ref as O


def _problem(seed=3, **kw):
    from orb_slam2_amd import synth
    return synth.fuse_problem(seed=seed, **kw)


def test_oracle_finds_planted_points():
    p = _problem()
    n, m = O.search_by_projection_sim3(p, 10.0)
    assert n > 0.3 * len(p["mp_xyz"]) and len(set(m[m >= 0].tolist())) == n


@pytest.mark.gpu
@pytest.mark.parametrize("seed,th", [(3, 10.0), (7, 5.0), (11, 15.0), (13, 60.0)])
def test_search_by_projection_sim3_gpu(amd, seed, th):
    from orb_slam2_amd import Frame
    p = _problem(seed)
    kf, kp = p["kf"], p["kp"]
    pre = np.full(len(kf["x"]), -1, np.int32)
    pre[np.random.default_rng(seed).random(len(pre)) < 0.1] = -2
    rn, rm = O.search_by_projection_sim3(p, th, pre)
    a = np.zeros(len(kf["x"]), dtype=[("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                                      ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
    a["x"], a["y"], a["octave"] = kf["x"], kf["y"], kf["octave"]
    fr = Frame(a, kf["desc"], kf["W"], kf["H"])
    m = amd.ORBmatcher(0.75, True)
    n, gm = m.SearchByProjectionSim3(fr, np.asarray(kp["Tcw"], np.float32)[:3, :4], kp["Ow"], kp["cam"],
                                     kp["log_scale_factor"], kp["scale_factors"], p["mp_valid"], p["mp_xyz"],
                                     p["mp_normal"], p["mp_min_dist"], p["mp_max_dist"], p["mp_desc"], th, pre)
    assert n == rn and np.array_equal(gm, rm) and n > 0
    m.close()
