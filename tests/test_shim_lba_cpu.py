"""The drop-in LocalBundleAdjustment's host side on the CPU: the compiled shim (tests/cpp/shim_caller.cpp,
mode `lbacpu`) gathers the window from mock keyframes / map points, builds the problem arrays and
writes the result back exactly as for the GPU, with the oracle's solve (oracle/lba_oracle.h) in place of
lba_solve.  Checked here, with no GPU:
  * the per-thread scratch and the host pool (ORB_SHIM_THREADS = 0, 1, 4, 7) give byte-identical
    outputs: gathered arrays, solve, erase log, written-back poses / points / observation counts;
  * the gathered graph and the vToErase order follow R/src/Optimizer.cpp:567-668, 850-880;
  * the solve equals the oracle's on the gathered arrays (bitwise: the same function)."""
import numpy as np
import pytest

import oracle_ref as O
from test_cpp_shim import _read, _run, shim  # noqa: F401  (shim: the compiled-caller fixture)

DT = (np.float64, np.float64, np.uint8, np.int64, np.float64, np.int64, np.uint8, np.int32, np.int32, np.uint8,
      np.float64, np.float64, np.float64, np.uint8, np.float64, np.float64, np.float64, np.int32, np.float32,
      np.float32, np.int32, np.int32, np.int64)


def _arrays(pb):
    inv_sigma2 = (np.float32(1.0) / np.array([np.float32(1.2) ** (2 * lv) for lv in range(8)], np.float32))
    octave = np.array([int(np.argmin(np.abs(inv_sigma2.astype(np.float64) - i))) for i in pb["edge_info"]], np.int32)
    return (np.asarray(pb["Tcw"], np.float32).reshape(-1), np.asarray(pb["pose_fixed"], np.uint8),
            np.asarray(pb["pose_id"], np.int64), np.asarray(pb["point_xyz"], np.float32).reshape(-1),
            np.asarray(pb["point_id"], np.int64), np.asarray(pb["edge_point"], np.int32),
            np.asarray(pb["edge_pose"], np.int32), np.asarray(pb["edge_obs"], np.float32).reshape(-1), octave,
            np.asarray(pb["edge_cam"][0], np.float32), inv_sigma2, np.zeros(1, np.uint8))


@pytest.mark.parametrize("stereo,outl", [(0.0, 0.0), (0.4, 0.2)])
def test_shim_lba_host_side_cpu(shim, tmp_path, monkeypatch, stereo, outl):  # noqa: F811
    from orb_slam2_amd import synth
    monkeypatch.setenv("ORB_ORACLE_LIB", str(O.LIB_PATH))
    pb = synth.ba_problem(n_local=8, n_fixed=3, n_points=700, stereo_frac=stereo, outlier_frac=outl, seed=17)
    outs = {}
    for t in (0, 1, 4, 7):
        monkeypatch.setenv("ORB_SHIM_THREADS", str(t))
        d = tmp_path / f"t{t}"
        d.mkdir()
        r, outp = _run(shim, "lbacpu", d, *_arrays(pb))
        assert r.returncode == 0, r.stderr
        outs[t] = outp.read_bytes()
    assert all(outs[t] == outs[0] for t in outs), "host pool changed the drop-in's outputs"
    (pq, pt, pfix, pid, X, xid, xbad, ept, eps, est, eobs, einfo, ecam, erase, oq, ot, ox, st, Tout, Xout, upd,
     nobs, elog) = _read(tmp_path / "t4" / "lbacpu.out", *DT)
    NP, NE = len(pfix), len(ept)
    e_pt, e_kf = np.asarray(pb["edge_point"]), np.asarray(pb["edge_pose"])
    fixed_in = np.asarray(pb["pose_fixed"])
    local_pts = np.unique(e_pt[fixed_in[e_kf] == 0])
    local_edge = np.isin(e_pt, local_pts)
    fixed_cams = np.unique(e_kf[local_edge & (fixed_in[e_kf] == 1)])
    local = np.nonzero(fixed_in == 0)[0]
    assert NP == len(local) + len(fixed_cams) and NE == int(local_edge.sum()) and len(xid) == len(local_pts)
    kf_of_pose = {int(i): k for k, i in enumerate(np.asarray(pb["pose_id"]))}
    Tcw = np.stack([np.asarray(pb["Tcw"], np.float32)[kf_of_pose[int(i)]] for i in pid])
    prob = dict(Tcw=Tcw, pose_fixed=pfix, pose_id=pid, point_xyz=X.reshape(-1, 3), point_id=xid, point_bad=xbad,
                edge_point=ept, edge_pose=eps, edge_stereo=est, edge_obs=eobs.reshape(-1, 3), edge_info=einfo,
                edge_cam=ecam.reshape(-1, 5))
    orc = O.lba_solve(prob)
    assert tuple(st[:2]) == orc["iterations"] and int(st[2]) == orc["trials"] and int(st[3]) == 0
    assert np.array_equal(erase, orc["edge_erase"])
    assert np.array_equal(oq.reshape(-1, 4), orc["pose_q"]) and np.array_equal(ox.reshape(-1, 3), orc["point_xyz"])
    mp_mnid = xid - (pid.max() + 1)
    want = [(int(pid[eps[e]]), int(mp_mnid[ept[e]])) for pas in (0, 1) for e in range(NE) if erase[e] and int(est[e]) == pas]
    assert [tuple(x) for x in elog.reshape(-1, 2)] == want
    if outl:
        assert erase.any()
    is_local = np.zeros(len(pb["point_id"]), bool)
    is_local[local_pts] = True
    assert np.array_equal(upd, is_local.astype(np.int32))
    nobs0 = np.bincount(e_pt, minlength=len(is_local))
    assert int(nobs.sum()) == int(nobs0.sum()) - int(erase.sum())
