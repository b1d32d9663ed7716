"""The OpenMP CPU path of local BA (g2o's G2O_OPENMP loops,
G/core/sparse_optimizer.cpp:70-71, G/core/block_solver.hpp:379-380, 528) keeps every sum in
the serial order, so it must reproduce the single-thread oracle bit for bit: the same LM
iterations / trials, chi2 trace, estimates and erase flags."""
import pathlib
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]


@pytest.mark.parametrize("kw", [dict(n_points=1500, seed=5), dict(n_points=1200, seed=21, stereo_frac=0.5)])
@pytest.mark.parametrize("threads", [2, 8])
def test_openmp_local_ba_bitwise_equal_to_serial(kw, threads):
    import pkgload
    pkgload.load()
    from orb_slam2_amd import synth
    import oracle_ref as O
    pb = synth.ba_problem(**kw)
    a = O.lba_solve(pb)
    b = O.lba_solve(pb, threads=threads)
    assert a["status"] == b["status"] == 0
    assert a["iterations"] == b["iterations"] and a["trials"] == b["trials"]
    for k in ("trace", "pose_q", "pose_t", "point_xyz", "edge_chi2", "edge_erase"):
        assert np.array_equal(a[k], b[k]), k
