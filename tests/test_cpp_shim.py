"""A compiled C++ caller of liborbslam2_amd (tests/cpp/shim_caller.cpp) through the class-surface
shim include/orbslam2_amd_shim.hpp, with mock cv::Mat / KeyPoint / Frame / KeyFrame / MapPoint /
Map types carrying the member names the reference's own types have:
  * CPU: the program compiles with -Wall -Wextra -Werror, links the library through the header,
    and without a GPU fails cleanly (exit 3, the ORB_ENODEV message) instead of falling back;
  * GPU: ORBextractor::operator(), ORBmatcher::SearchForInitialization and both tracking forms of
    ORBmatcher::SearchByProjection through the shim are bit-exact against the oracle;
    Optimizer::LocalBundleAdjustment through the shim gathers the reference's graph
    (R/src/Optimizer.cpp:567-782) from the mock keyframes, solves within the oracle's tolerances
    (identical LM decisions and erase set, poses / points to 1e-5), and writes back (:850-917)
    exactly what lba_solve returns, erasing mono observations before stereo ones."""
import os
import pathlib
import shutil
import subprocess

import numpy as np
import pytest

import oracle_ref as O
from test_matcher_gpu import _sbp_setup

ROOT = pathlib.Path(__file__).resolve().parents[1]
LIB_DIR = ROOT / "orb-slam2-_amd" / "lib"


@pytest.fixture(scope="module")
def shim(tmp_path_factory):
    if os.environ.get("ORB_SHIM_CALLER"):   # a prebuilt caller (tools/sanitize_cpu.sh: the ASan/UBSan build)
        return pathlib.Path(os.environ["ORB_SHIM_CALLER"])
    gxx = shutil.which("g++")
    if gxx is None or not (LIB_DIR / "liborbslam2_amd.so").exists():
        pytest.skip("g++ or the built library is missing")
    exe = tmp_path_factory.mktemp("shim") / "shim_caller"
    # -ffp-contract=off: the build flag INTEGRATION.md asks of the drop-in, so the shim's
    # few float expressions (the triangulation epipole) round as the oracle's do
    subprocess.run([gxx, "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", "-ffp-contract=off", "-pthread",
                    f"-I{ROOT / 'include'}",
                    str(ROOT / "tests" / "cpp" / "shim_caller.cpp"), f"-L{LIB_DIR}", "-lorbslam2_amd",
                    f"-Wl,-rpath,{LIB_DIR}", "-o", str(exe)], check=True, capture_output=True, text=True)
    return exe


def _write(path, *arrays):
    with open(path, "wb") as f:
        for a in arrays:
            a = np.ascontiguousarray(a)
            np.array([a.size], np.int64).tofile(f)
            a.tofile(f)


def _read(path, *dtypes):
    out = []
    with open(path, "rb") as f:
        for dt in dtypes:
            n = int(np.fromfile(f, np.int64, 1)[0])
            out.append(np.fromfile(f, dt, n))
    return out


def _run(exe, mode, tmp_path, *arrays):
    inp, outp = tmp_path / f"{mode}.in", tmp_path / f"{mode}.out"
    _write(inp, *arrays)
    r = subprocess.run([str(exe), mode, str(inp), str(outp)], capture_output=True, text=True, timeout=120)
    return r, outp


def test_shim_builds_and_fails_cleanly_without_gpu(shim, tmp_path):
    """Without a usable gfx950 device (this container) the shim's constructors throw: the program
    reports the library's ORB_ENODEV status and exits 3, no CPU fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: covered by the gpu tests")
    img = np.zeros((480, 640), np.uint8)
    r, _ = _run(shim, "extract", tmp_path, np.array([640, 480, 1000], np.int32), img)
    assert r.returncode == 3 and "failed (-19)" in r.stderr, (r.returncode, r.stderr)
    T = np.tile(np.eye(4, dtype=np.float32).reshape(-1), 2)     # two local keyframes, one point
    r, _ = _run(shim, "lba", tmp_path, T, np.zeros(2, np.uint8), np.array([0, 1], np.int64),
                np.array([0, 0, 5], np.float32), np.array([7], np.int64), np.zeros(2, np.int32),
                np.array([0, 1], np.int32), np.array([320, 240, -1, 321, 240, -1], np.float32),
                np.zeros(2, np.int32), np.array([500, 500, 320, 240, 0], np.float32), np.ones(8, np.float32),
                np.zeros(1, np.uint8))
    assert r.returncode == 3 and "failed (-19)" in r.stderr, (r.returncode, r.stderr)


@pytest.mark.gpu
def test_shim_extract_matches_oracle(shim, tmp_path):
    from orb_slam2_amd import synth
    cv = synth.canvas(0x5EED0001, 640, 480)
    img = synth.frame(cv, 640, 480, 3)
    r, outp = _run(shim, "extract", tmp_path, np.array([640, 480, 1000], np.int32), img)
    assert r.returncode == 0, r.stderr
    kb, desc, sizes, sf = _read(outp, np.uint8, np.uint8, np.int32, np.float32)
    kps = kb.view(O.KP_DTYPE)
    ref = O.extract(O.params(1000), img)
    assert np.array_equal(kps, ref["kps"]) and np.array_equal(desc.reshape(-1, 32), ref["desc"])
    lw, lh = O.level_sizes(O.params(1000), 640, 480)
    assert np.array_equal(sizes.reshape(-1, 2), np.stack([lw, lh], 1))
    assert np.array_equal(sf, O.tables(O.params(1000))["scale"])


@pytest.mark.gpu
def test_shim_search_for_initialization_matches_oracle(shim, tmp_path):
    from orb_slam2_amd import synth
    cv = synth.canvas(0x5EED0002, 640, 480)
    p = O.params(1000)
    a, b = O.extract(p, synth.frame(cv, 640, 480, 0)), O.extract(p, synth.frame(cv, 640, 480, 1))
    prev = np.stack([a["kps"]["x"], a["kps"]["y"]], 1).astype(np.float32).reshape(-1)
    fa, fb = O.FrameView(a["kps"], a["desc"], 640, 480), O.FrameView(b["kps"], b["desc"], 640, 480)
    n_ref, m_ref, prev_ref = O.search_for_initialization(fa, fb, prev.copy(), nnratio=0.9, window=100)

    def frame(e):
        k = e["kps"]
        return (np.ascontiguousarray(k["x"], np.float32), np.ascontiguousarray(k["y"], np.float32),
                np.ascontiguousarray(k["angle"], np.float32), np.ascontiguousarray(k["octave"], np.int32),
                np.ascontiguousarray(e["desc"], np.uint8))
    grid = np.array([0, 0, 640, 480, np.float32(64) / np.float32(640), np.float32(48) / np.float32(480)], np.float32)
    r, outp = _run(shim, "sfi", tmp_path, *frame(a), *frame(b), grid, prev, np.array([100], np.int32))
    assert r.returncode == 0, r.stderr
    n, m12, prev_out, d01 = _read(outp, np.int32, np.int32, np.float32, np.int32)
    assert int(n[0]) == n_ref and np.array_equal(m12, m_ref) and np.array_equal(prev_out, prev_ref)
    assert int(d01[0]) == O.descriptor_distance(a["desc"][0], b["desc"][0])


def _frame_arrays(kps, desc):
    return (np.ascontiguousarray(kps["x"], np.float32), np.ascontiguousarray(kps["y"], np.float32),
            np.ascontiguousarray(kps["angle"], np.float32), np.ascontiguousarray(kps["octave"], np.int32),
            np.ascontiguousarray(desc, np.uint8))


GRID = np.array([0, 0, 640, 480, np.float32(64) / np.float32(640), np.float32(48) / np.float32(480)], np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("stereo,th,temporal", [(False, 15.0, False), (True, 7.0, True)])
def test_shim_search_by_projection_frame_matches_oracle(shim, tmp_path, stereo, th, temporal):
    """Tracking::TrackWithMotionModel's call through the shim: the mock frames' mTcw, mvpMapPoints
    (with and without observations), mvbOutlier, mvuRight and the static intrinsics are gathered by
    the shim; CurrentFrame.mvpMapPoints comes back as the oracle's R :1564-1718 leaves it."""
    a, b, cam, xyz, Tl, Tc, has, outl, mpd, ur, sf = _sbp_setup(stereo=stereo)
    init = np.full(len(b["kps"]), -1, np.int32)
    init[::17] = -2
    if temporal:
        rng = np.random.default_rng(12)
        has = np.where((has > 0) & (rng.random(len(has)) < 0.4), 2, has).astype(np.int32)
        init[5::19] = -3
    cur = O.FrameView(b["kps"], b["desc"], 640, 480, uright=ur)
    last = O.FrameView(a["kps"], a["desc"], 640, 480)
    n_ref, mp_ref = O.search_by_projection_ff(cur, Tc[:3], last, Tl[:3], has, outl, xyz, mpd, sf,
                                              O.Camera(*[float(v) for v in cam]), th, not stereo, True, init)
    urc = ur if ur is not None else np.full(len(b["kps"]), -1, np.float32)
    r, outp = _run(shim, "sbp", tmp_path, *_frame_arrays(b["kps"], b["desc"]), urc,
                   *_frame_arrays(a["kps"], a["desc"]), GRID, np.asarray(Tc, np.float32).reshape(-1),
                   np.asarray(Tl, np.float32).reshape(-1), has.astype(np.int32), outl.astype(np.uint8),
                   xyz.astype(np.float32).reshape(-1), mpd, sf.astype(np.float32), cam.astype(np.float32),
                   np.array([th], np.float32), np.array([0 if stereo else 1], np.int32), init)
    assert r.returncode == 0, r.stderr
    n, slots = _read(outp, np.int32, np.int32)
    assert int(n[0]) == n_ref and np.array_equal(slots, mp_ref)
    assert n_ref > 100


@pytest.mark.gpu
def test_shim_search_by_projection_local_matches_oracle(shim, tmp_path):
    """Tracking::SearchLocalPoints's call through the shim: mbTrackInView / isBad / mTrackProj* /
    mnTrackScaleLevel / mTrackViewCos / GetDescriptor / Observations read from mock map points."""
    from test_matcher_gpu import _sbl_setup
    b, in_view, proj, level, vcos, md, has_obs, ur, init, sf = _sbl_setup(stereo=True)
    f = O.FrameView(b["kps"], b["desc"], 640, 480, uright=ur)
    th = 3.0
    rng = np.random.default_rng(4)
    bad = (rng.random(len(in_view)) < 0.05) & in_view
    n_ref, mp_ref = O.search_by_projection_local(f, in_view & ~bad, proj, level, vcos, md, has_obs, sf, 0.8, th, init)
    r, outp = _run(shim, "sbl", tmp_path, *_frame_arrays(b["kps"], b["desc"]), ur, GRID,
                   in_view.astype(np.uint8), bad.astype(np.uint8), proj.astype(np.float32).reshape(-1),
                   level.astype(np.int32), vcos.astype(np.float32), md, has_obs.astype(np.uint8), sf.astype(np.float32),
                   np.array([th], np.float32), np.array([0.8], np.float32), init)
    assert r.returncode == 0, r.stderr
    n, slots = _read(outp, np.int32, np.int32)
    assert int(n[0]) == n_ref and np.array_equal(slots, mp_ref)
    assert n_ref > 50


@pytest.mark.gpu
@pytest.mark.parametrize("stereo,group", [(0.0, None), (0.4, None), (0.4, 2)])
def test_shim_local_bundle_adjustment(shim, tmp_path, amd, stereo, group):
    """group: the device-list overload (lba_group over `group` contexts, sharing the device on a
    one-GPU machine) — the same gathering and write-back, the same LM decisions."""
    from orb_slam2_amd import synth
    pb = synth.ba_problem(n_local=8, n_fixed=3, n_points=900, stereo_frac=stereo, seed=11)
    inv_sigma2 = (np.float32(1.0) / np.array([np.float32(1.2) ** (2 * l) for l in range(8)], np.float32))
    octave = np.array([int(np.argmin(np.abs(inv_sigma2.astype(np.float64) - i))) for i in pb["edge_info"]], np.int32)
    nk = len(pb["Tcw"])
    cam = np.asarray(pb["edge_cam"][0], np.float32)
    extra = []
    if group:
        import torch
        extra = [np.array([r % torch.cuda.device_count() for r in range(group)], np.int32)]
    r, outp = _run(shim, "lbag" if group else "lba", tmp_path, np.asarray(pb["Tcw"], np.float32).reshape(-1),
                   np.asarray(pb["pose_fixed"], np.uint8), np.asarray(pb["pose_id"], np.int64),
                   np.asarray(pb["point_xyz"], np.float32).reshape(-1), np.asarray(pb["point_id"], np.int64),
                   np.asarray(pb["edge_point"], np.int32), np.asarray(pb["edge_pose"], np.int32),
                   np.asarray(pb["edge_obs"], np.float32).reshape(-1), octave, cam, inv_sigma2,
                   np.zeros(1, np.uint8), *extra)
    assert r.returncode == 0, r.stderr
    (pq, pt, pfix, pid, X, xid, xbad, ept, eps, est, eobs, einfo, ecam, erase, oq, ot, ox, st, Tout, Xout, upd,
     nobs, elog) = _read(outp, np.float64, np.float64, np.uint8, np.int64, np.float64, np.int64, np.uint8, np.int32,
                         np.int32, np.uint8, np.float64, np.float64, np.float64, np.uint8, np.float64, np.float64,
                         np.float64, np.int32, np.float32, np.float32, np.int32, np.int32, np.int64)
    NP, NE = len(pfix), len(ept)
    # the gathered graph (R :567-668): the local points are those a local keyframe observes; every
    # observation of a local point is an edge; the fixed cameras are the other keyframes observing
    # one; ids as the reference assigns them (points: mnId + maxKFid + 1)
    e_pt, e_kf = np.asarray(pb["edge_point"]), np.asarray(pb["edge_pose"])
    fixed_in = np.asarray(pb["pose_fixed"])
    local_pts = np.unique(e_pt[fixed_in[e_kf] == 0])
    local_edge = np.isin(e_pt, local_pts)
    fixed_cams = np.unique(e_kf[local_edge & (fixed_in[e_kf] == 1)])
    local = np.nonzero(fixed_in == 0)[0]
    assert NP == len(local) + len(fixed_cams) and NE == int(local_edge.sum()) and len(xid) == len(local_pts)
    assert np.array_equal(pid[:len(local)], np.asarray(pb["pose_id"])[local])
    assert np.array_equal(np.sort(pid[len(local):]), np.sort(np.asarray(pb["pose_id"])[fixed_cams]))
    assert np.array_equal(pfix[len(local):], np.ones(NP - len(local), np.uint8))
    assert np.array_equal(np.sort(xid - (pid.max() + 1)), np.sort(np.asarray(pb["point_id"])[local_pts]))
    # the same arrays through the Python binding of lba_solve: bitwise the same solve
    kf_of_pose = {int(i): k for k, i in enumerate(np.asarray(pb["pose_id"]))}
    Tcw = np.stack([np.asarray(pb["Tcw"], np.float32)[kf_of_pose[int(i)]] for i in pid])
    prob = dict(Tcw=Tcw, pose_fixed=pfix, pose_id=pid, point_xyz=X.reshape(-1, 3), point_id=xid, point_bad=xbad,
                edge_point=ept, edge_pose=eps, edge_stereo=est, edge_obs=eobs.reshape(-1, 3), edge_info=einfo,
                edge_cam=ecam.reshape(-1, 5))
    ref = amd.LocalBA().solve(prob)
    assert tuple(st[:2]) == ref["iterations"] and int(st[2]) == ref["trials"] and int(st[3]) == 0
    if group:   # sharded sums: the same decisions, estimates to rounding; compare with the group solve
        ref = amd.LocalBAGroup(extra[0].tolist()).solve(prob)
    # ... and within the oracle's tolerances (tests/test_lba_gpu.py): same LM decisions, same erase set
    orc = O.lba_solve(prob)
    assert tuple(st[:2]) == orc["iterations"] and int(st[2]) == orc["trials"]
    assert np.array_equal(erase, orc["edge_erase"])
    assert np.abs(oq.reshape(-1, 4) - orc["pose_q"]).max() < 1e-5 and np.abs(ot.reshape(-1, 3) - orc["pose_t"]).max() < 1e-5
    assert np.abs(ox.reshape(-1, 3) - orc["point_xyz"]).max() < 1e-5
    # vToErase order (R :850-880): every erased mono edge in edge order, then every erased stereo edge
    mp_mnid = xid - (pid.max() + 1)
    want = [(int(pid[eps[e]]), int(mp_mnid[ept[e]])) for pas in (0, 1) for e in range(NE)
            if erase[e] and int(est[e]) == pas]
    assert [tuple(x) for x in elog.reshape(-1, 2)] == want
    if stereo:
        assert erase[est == 1].any() and erase[est == 0].any()
    assert np.array_equal(oq.reshape(-1, 4), ref["pose_q"]) and np.array_equal(ot.reshape(-1, 3), ref["pose_t"])
    assert np.array_equal(ox.reshape(-1, 3), ref["point_xyz"]) and np.array_equal(erase, ref["edge_erase"])
    # write-back (R :883-917): local keyframes' Tcw = Converter::toCvMat of the estimate, fixed
    # cameras untouched, every point moved and UpdateNormalAndDepth'ed once, erased observations gone
    from orb_slam2_amd import optimizer as opt
    for k in range(len(local)):
        assert np.array_equal(Tout.reshape(nk, 4, 4)[kf_of_pose[int(pid[k])]],
                              opt.pose_to_Tcw(ref["pose_q"][k], ref["pose_t"][k]))
    is_local = np.zeros(len(pb["point_id"]), bool)
    is_local[local_pts] = True
    assert np.array_equal(upd, is_local.astype(np.int32))    # points outside the window untouched
    nobs0 = np.bincount(e_pt, minlength=len(is_local))
    assert int(nobs.sum()) == int(nobs0.sum()) - int(erase.sum())
    assert np.array_equal(nobs[~is_local], nobs0[~is_local])
