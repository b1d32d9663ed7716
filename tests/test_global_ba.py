"""Optimizer::BundleAdjustment (global BA, R/src/Optimizer.cpp:78-277) — the local-BA kernels run
as one optimize(nIterations) over every keyframe and map point, Huber kernels only with bRobust,
no outlier pass.  CPU: oracle properties; GPU: the same LM decisions as the oracle, chi2 to 1e-9
relative, poses / points to 1e-5 (north_star tolerance)."""
import ctypes as C

import numpy as np
import pytest

import oracle_ref as O


def _problem(extra_unobserved=0, **kw):
    from orb_slam2_amd import synth
    pb = synth.ba_problem(**kw)
    if extra_unobserved:   # map points with no edge: left out (vbNotIncludedMP), returned unchanged
        n = len(pb["point_xyz"])
        pb["point_xyz"] = np.concatenate([pb["point_xyz"], np.full((extra_unobserved, 3), 3.0)])
        pb["point_id"] = np.concatenate([pb["point_id"], pb["point_id"].max() + 1 + np.arange(extra_unobserved)])
        pb["point_bad"] = np.concatenate([pb["point_bad"], np.zeros(extra_unobserved, pb["point_bad"].dtype)])
        assert len(pb["point_xyz"]) == n + extra_unobserved
    return pb


def _chi2(ref):
    return ref["trace"][:, 1]


def test_oracle_global_ba_properties():
    pb = _problem(n_local=10, n_fixed=0, n_points=800, seed=4, extra_unobserved=3)
    r = O.global_ba(pb, 10, robust=False)
    assert r["iterations"][1] == 0 and not r["edge_erase"].any()
    assert _chi2(r)[-1] < r["trace"][0, 0]                          # the optimisation reduces chi2
    assert np.array_equal(r["point_xyz"][-3:], np.full((3, 3), 3.0))
    rr = O.global_ba(pb, 10, robust=True)
    assert not np.allclose(rr["pose_t"], r["pose_t"])               # Huber changes the solution
    s = O.global_ba(pb, 10, robust=False, stop=True)                # force stop: no iteration, written
    assert s["status"] == 0 and s["iterations"] == (0, 0)
    assert np.allclose(s["point_xyz"], pb["point_xyz"])


def _compare(ref, got, tol=1e-5):
    assert got["iterations"] == ref["iterations"], (got["iterations"], ref["iterations"])
    assert got["trials"] == ref["trials"]
    for k in range(3):
        assert np.allclose(got["trace"][:, k], ref["trace"][:, k], rtol=1e-9, atol=0)
    assert np.abs(got["pose_q"] - ref["pose_q"]).max() < tol
    assert np.abs(got["pose_t"] - ref["pose_t"]).max() < tol
    assert np.abs(got["point_xyz"] - ref["point_xyz"]).max() < tol
    assert not got["edge_erase"].any()
    assert np.allclose(got["edge_chi2"], ref["edge_chi2"], rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("kw,robust,iters", [
    (dict(n_local=20, n_fixed=0, n_points=3000), False, 10),          # LoopClosing: 10 its, bRobust false
    (dict(n_local=12, n_fixed=0, n_points=1500, stereo_frac=0.5, seed=7), True, 20),   # initialisation: 20
    (dict(n_local=40, n_fixed=0, n_points=5000, seed=13, extra_unobserved=5), False, 10),   # 6P = 240 > LDS
])
def test_global_ba_matches_oracle(amd, kw, robust, iters):
    pb = _problem(**kw)
    ref = O.global_ba(pb, iters, robust=robust)
    got = amd.Optimizer.BundleAdjustment(pb, iters, bRobust=robust)
    _compare(ref, got)


@pytest.mark.gpu
def test_global_ba_stop_flag_writes_back(amd):
    pb = _problem(n_local=8, n_fixed=0, n_points=400, seed=2)
    flag = (C.c_uint8 * 1)(1)
    got = amd.Optimizer.BundleAdjustment(pb, 10, pbStopFlag=flag, bRobust=False)
    ref = O.global_ba(pb, 10, robust=False, stop=True)
    assert not got["aborted"] and got["iterations"] == (0, 0)
    _compare(ref, got)
