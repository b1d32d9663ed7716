"""The relocalisation and loop-closing rows of SURVEY §8f through the compiled C++ drop-in path
(tests/cpp/shim_caller.cpp over include/orbslam2_amd_shim.hpp, mock reference types), bit-exact
against the oracle:

* ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
  (R/src/ORBmatcher.cpp:1719-1800, Tracking::Relocalization): the shim derives Ow from mTcw and
  drops NULL / bad / sAlreadyFound points; pre-set frame slots stay;
* SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (:370-497) and Fuse(pKF, Scw, vpPoints,
  th, vpReplacePoint) (:1164-1290), LoopClosing::ComputeSim3 / SearchAndFuse: the shim removes
  the Sim3 scale from Scw (detail::decompose_scw, restated below), skips bad points and those
  already matched / already in the keyframe, and resolves Fuse's replace / add step in vector
  order (checked against a Python restatement of :1263-1283 driven by the oracle's matches);
* SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (:1305-1503): the shim forms sR12,
  sR21, t21 and vbAlreadyMatched1 / 2 (through GetIndexInKeyFrame) from a partly filled
  vpMatches12."""
import numpy as np
import pytest

import oracle_ref as O
from test_cpp_shim import GRID, _frame_arrays, _read, _run, shim  # noqa: F401  (fixture)
from test_cpp_shim_dropin import EMPTY_FV, ISG2, SF, SG2, _kf_arrays

pytestmark = pytest.mark.gpu
F32 = np.float32


def _center(T):
    """Ow = -R^T t as the shim evaluates it (double accumulation in row order, one rounding)."""
    T = np.asarray(T, np.float64)
    return np.array([-(T[0, k] * T[0, 3] + T[1, k] * T[1, 3] + T[2, k] * T[2, 3]) for k in range(3)]).astype(F32)


def _decompose_scw(Scw):
    """R/src/ORBmatcher.cpp:382-386 as the shim evaluates it: scw = sqrt(row0 . row0) in double,
    rounded to float; each element times 1.0 / scw in double, rounded once; Ow = -R^T t."""
    S = np.asarray(Scw, F32)
    ss = 0.0
    for k in range(3):
        v = float(S[0, k])
        ss += v * v
    inv = 1.0 / float(F32(np.sqrt(ss)))
    T = (S[:3, :4].astype(np.float64) * inv).astype(F32)
    return T, _center(T)


def _scw(kp, s):
    S = np.eye(4, dtype=F32)
    S[:3, :4] = (np.asarray(kp["Tcw"], F32)[:3, :4].astype(np.float64) * s).astype(F32)
    return S


def _pts(xyz, nrm, mind, maxd, desc):
    return (np.asarray(xyz, F32).reshape(-1), np.asarray(nrm, F32).reshape(-1), np.asarray(mind, F32),
            np.asarray(maxd, F32), np.ascontiguousarray(desc, np.uint8).reshape(-1))


# ------------------------------------------------------------------ relocalisation
@pytest.mark.parametrize("seed,th,orb_dist,ori", [(3, 10.0, 100, True), (4, 10.0, 100, True), (5, 5.0, 64, False)])
def test_shim_search_by_projection_keyframe(shim, tmp_path, seed, th, orb_dist, ori):
    from test_sbp_kf import _problem
    p, kf, kfs, occ = _problem(seed)
    kp = p["kp"]
    rng = np.random.default_rng(seed + 7)
    n_mp = len(p["mp_xyz"])
    # keyframe slots: -1 no point, 0 good, 1 bad, 2 good but in sAlreadyFound
    kind = np.where(p["mp_valid"] != 0, 0, rng.choice([-1, 1, 2], n_mp)).astype(np.int32)
    kind[(kind == 0) & (rng.random(n_mp) < 0.05)] = 2
    T = np.eye(4, dtype=F32)
    T[:3, :4] = np.asarray(kp["Tcw"], F32)[:3, :4]
    cam4 = np.asarray(kp["cam"][:4], F32)
    kfa = _kf_arrays(kfs, np.eye(4, dtype=F32), np.zeros(3, F32), np.append(cam4, F32(0)), SF, ISG2, SG2, EMPTY_FV)
    r, outp = _run(shim, "sbpk", tmp_path, *_frame_arrays(kf, kf["desc"]), GRID, T.reshape(-1), cam4,
                   np.array([kp["log_scale_factor"]], F32), np.asarray(kp["scale_factors"], F32), occ, *kfa, kind,
                   *_pts(p["mp_xyz"], p["mp_normal"], p["mp_min_dist"], p["mp_max_dist"], p["mp_desc"]),
                   np.array([th, orb_dist, float(ori)], F32))
    assert r.returncode == 0, r.stderr
    n, slots = _read(outp, np.int32, np.int32)
    cur = O.FrameView(kf, kf["desc"], kf["W"], kf["H"])
    kv = O.FrameView(kfs, kfs["desc"], kfs["W"], kfs["H"])
    rn, rm = O.search_by_projection_kf(cur, T[:3, :4], _center(T[:3]), kv, (kind == 0).astype(np.uint8), p["mp_xyz"],
                                       p["mp_min_dist"], p["mp_max_dist"], p["mp_desc"], cam4, kp["log_scale_factor"],
                                       kp["scale_factors"], th, orb_dist, ori, occ)
    assert int(n[0]) == rn and np.array_equal(slots, rm) and rn > 50
    assert np.all(slots[occ == -2] == -2)


# ------------------------------------------------------------------ loop closing, Scw forms
@pytest.mark.parametrize("seed,th,s", [(3, 10, 1.0), (7, 5, 1.25), (11, 15, 0.8)])
def test_shim_search_by_projection_scw(shim, tmp_path, seed, th, s):
    from orb_slam2_amd import synth
    p = synth.fuse_problem(seed=seed)
    kf, kp = p["kf"], p["kp"]
    rng = np.random.default_rng(seed + 3)
    nk, nm = len(kf["x"]), len(p["mp_xyz"])
    # the points the problem marks invalid: half bad, half already in vpMatched; a few foreign
    # points fill other slots
    inval = np.flatnonzero(p["mp_valid"] == 0)
    bad = np.zeros(nm, np.uint8)
    bad[inval[: len(inval) // 2]] = 1
    placed = inval[len(inval) // 2:]
    pre = np.full(nk, -1, np.int32)
    slots = rng.choice(nk, len(placed) + 40, replace=False)
    pre[slots[: len(placed)]] = placed
    pre[slots[len(placed):]] = -2
    Scw = _scw(kp, s)
    Tdec, Owdec = _decompose_scw(Scw)
    kfa = _kf_arrays(kf, np.eye(4, dtype=F32), np.zeros(3, F32), kp["cam"], kp["scale_factors"], kp["inv_level_sigma2"],
                     SG2, EMPTY_FV)
    r, outp = _run(shim, "sbps", tmp_path, *kfa, Scw.reshape(-1), bad,
                   *_pts(p["mp_xyz"], p["mp_normal"], p["mp_min_dist"], p["mp_max_dist"], p["mp_desc"]), pre,
                   np.array([th], np.int32))
    assert r.returncode == 0, r.stderr
    n, got = _read(outp, np.int32, np.int32)
    q = dict(p, kp=dict(kp, Tcw=Tdec, Ow=Owdec))
    rn, rm = O.search_by_projection_sim3(q, float(th), np.where(pre == -1, -1, -2).astype(np.int32))
    assert int(n[0]) == rn and rn > 50
    assert np.array_equal(got, np.where(rm >= 0, rm, pre))


def _py_fuse_scw_resolve(best, vec, n_slots, slot0, bad):
    """R/src/ORBmatcher.cpp:1263-1283 in vector order: the keyframe's point in the matched slot
    (as the loop finds it) becomes vpReplacePoint unless bad; an empty slot takes the point."""
    slots = [-1] * n_slots
    in_kf = [int(x) for x in slot0]
    for i, x in enumerate(slot0):
        if x >= 0:
            slots[x] = i
    repl = [-1] * len(vec)
    n = 0
    for j, v in enumerate(vec):
        b = int(best[v])
        if b < 0:
            continue
        q = slots[b]
        if q >= 0:
            if not bad[q]:
                repl[j] = q
        else:
            slots[b], in_kf[v] = v, b
        n += 1
    return n, slots, repl, in_kf


@pytest.mark.parametrize("seed,th,s", [(3, 4.0, 1.0), (9, 4.0, 1.4)])
def test_shim_fuse_scw(shim, tmp_path, seed, th, s):
    from orb_slam2_amd import synth
    p = synth.fuse_problem(seed=seed)
    kf, kp = p["kf"], p["kp"]
    rng = np.random.default_rng(seed + 5)
    nk, nm = len(kf["x"]), len(p["mp_xyz"])
    own = np.flatnonzero(rng.random(nk) < 0.3)          # the keyframe's own points (zero data)
    n_own = len(own)
    np_ = nm + n_own
    inval = np.flatnonzero(p["mp_valid"] == 0)
    bad = np.zeros(np_, np.uint8)
    bad[inval[: len(inval) // 2]] = 1
    bad[nm:] = rng.random(n_own) < 0.15                 # some of the keyframe's points are bad
    slot = np.full(np_, -1, np.int32)
    free = np.setdiff1d(np.arange(nk), own)
    slot[inval[len(inval) // 2:]] = rng.choice(free, len(inval) - len(inval) // 2, replace=False)
    slot[nm:] = own
    vec = list(range(nm)) + [int(i) for i in rng.choice(n_own, 30, replace=False) + nm]
    vec += [int(i) for i in rng.choice(np.flatnonzero(p["mp_valid"] != 0), 25, replace=False)]   # repeats
    rng.shuffle(vec)
    pad = lambda a, w: np.concatenate([np.asarray(a, F32).reshape(nm, -1), np.zeros((n_own, w), F32)]).reshape(-1)
    desc = np.concatenate([p["mp_desc"], np.zeros((n_own, 32), np.uint8)])
    Scw = _scw(kp, s)
    Tdec, Owdec = _decompose_scw(Scw)
    kfa = _kf_arrays(kf, np.eye(4, dtype=F32), np.zeros(3, F32), kp["cam"], kp["scale_factors"], kp["inv_level_sigma2"],
                     SG2, EMPTY_FV)
    r, outp = _run(shim, "fuses", tmp_path, *kfa, Scw.reshape(-1), bad,
                   *_pts(pad(p["mp_xyz"], 3), pad(p["mp_normal"], 3), pad(p["mp_min_dist"], 1),
                         pad(p["mp_max_dist"], 1), desc), slot, np.array(vec, np.int32), np.array([th], F32))
    assert r.returncode == 0, r.stderr
    n, slots, repl, po = _read(outp, np.int32, np.int32, np.int32, np.int32)
    # the matching step: the oracle on the points valid at entry (not bad, not in the keyframe)
    q = dict(p, kp=dict(kp, Tcw=Tdec, Ow=Owdec),
             mp_valid=((bad[:nm] == 0) & (slot[:nm] < 0)).astype(np.uint8))
    best, _ = O.fuse(q, th, sim3=True)
    best_all = np.full(np_, -1, np.int32)
    best_all[:nm] = best
    rn, rslots, rrepl, rin = _py_fuse_scw_resolve(best_all, vec, nk, slot, bad)
    assert int(n[0]) == rn and rn > 100
    assert np.array_equal(slots, rslots) and np.array_equal(repl, rrepl) and np.array_equal(po, rin)
    assert (repl >= 0).sum() > 10 and (repl[np.array(vec) >= nm] < 0).all()


# ------------------------------------------------------------------ SearchBySim3
@pytest.mark.parametrize("seed,s12,th", [(6, 1.0, 7.5), (8, 1.03, 7.5), (9, 0.97, 4.0)])
def test_shim_search_by_sim3(shim, tmp_path, seed, s12, th):
    from orb_slam2_amd import synth
    p = synth.sim3_problem(seed=seed, s12=s12)
    k1, k2 = p["kf1"], p["kf2"]
    rng = np.random.default_rng(seed + 11)
    kinds, ins = [], []
    for k in (k1, k2):
        kind = np.where(k["mp_valid"] != 0, 0, -1).astype(np.int32)
        kind[(kind == 0) & (rng.random(len(kind)) < 0.08)] = 1
        kinds.append(kind)
        T = np.eye(4, dtype=F32)
        T[:3, :4] = k["Tcw"]
        cam = np.array(list(p["cam"]) + [0.0], F32)
        ins += [*_kf_arrays(k, T, _center(T[:3]), cam, p["scale_factors"], ISG2, SG2, EMPTY_FV), kind,
                *_pts(k["mp_xyz"], np.zeros(0, F32), k["mp_min_dist"], k["mp_max_dist"], k["mp_desc"])]
    n1, n2 = len(k1["x"]), len(k2["x"])
    # vpMatches12 on entry: some keyframe-1 slots already hold a keyframe-2 point, a few a point
    # keyframe 2 does not observe
    pre = np.full(n1, -1, np.int32)
    c1 = rng.choice(np.flatnonzero(kinds[0] == 0), 30, replace=False)
    pre[c1[:24]] = rng.choice(np.flatnonzero(kinds[1] >= 0), 24, replace=False)
    pre[c1[24:]] = -2
    r, outp = _run(shim, "sbs", tmp_path, *ins, pre, np.array([p["s12"]], F32), np.asarray(p["R12"], F32).reshape(-1),
                   np.asarray(p["t12"], F32), np.array([th], F32))
    assert r.returncode == 0, r.stderr
    n, got = _read(outp, np.int32, np.int32)
    am2 = np.zeros(n2, bool)
    am2[pre[pre >= 0]] = True
    q = dict(p, kf1=dict(k1, mp_valid=((kinds[0] == 0) & (pre == -1)).astype(np.uint8)),
             kf2=dict(k2, mp_valid=((kinds[1] == 0) & ~am2).astype(np.uint8)))
    rn, rm = O.search_by_sim3(q, th)
    assert int(n[0]) == rn and rn > 50
    assert np.array_equal(got, np.where(pre != -1, pre, rm))
