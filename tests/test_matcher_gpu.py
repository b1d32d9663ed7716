"""GPU matcher parity vs the CPU oracle (bit-exact match indices and counts)."""
import numpy as np
import pytest

import oracle_ref as O

pytestmark = pytest.mark.gpu


def _pair(W, H, seed, nf, t=0, dt=1):
    from orb_slam2_amd import synth
    cv = synth.canvas(seed, W, H)
    p = O.params(nf)
    a = O.extract(p, synth.frame(cv, W, H, t))
    b = O.extract(p, synth.frame(cv, W, H, t + dt))
    return a, b


@pytest.mark.parametrize("W,H,nf,seed,window,nn", [
    (640, 480, 1000, 0x5EED0001, 100, 0.9),
    (640, 480, 2000, 0x5EED0002, 100, 0.9),
    (640, 480, 1000, 0x5EED0007, 10, 0.6),
    (1241, 376, 2000, 0x5EED0003, 100, 0.9),
])
def test_search_for_initialization(amd, W, H, nf, seed, window, nn):
    a, b = _pair(W, H, seed, nf)
    F1 = amd.Frame(a["kps"], a["desc"], W, H)
    F2 = amd.Frame(b["kps"], b["desc"], W, H)
    prev = np.stack([a["kps"]["x"], a["kps"]["y"]], 1).astype(np.float32)
    fa, fb = O.FrameView(a["kps"], a["desc"], W, H), O.FrameView(b["kps"], b["desc"], W, H)
    n_ref, m_ref, prev_ref = O.search_for_initialization(fa, fb, prev.reshape(-1), nnratio=nn, window=window)
    m = amd.ORBmatcher(nn, True)
    prev_gpu = prev.copy()
    n, m12 = m.SearchForInitialization(F1, F2, prev_gpu, window)
    assert n == n_ref
    assert np.array_equal(m12, m_ref)
    assert np.array_equal(prev_gpu.reshape(-1), prev_ref)
    if window == 100:
        assert n > 50   # the synthetic pair really matches


def test_search_for_initialization_no_orientation_check(amd):
    a, b = _pair(640, 480, 0x5EED0001, 1000)
    fa, fb = O.FrameView(a["kps"], a["desc"], 640, 480), O.FrameView(b["kps"], b["desc"], 640, 480)
    prev = np.stack([a["kps"]["x"], a["kps"]["y"]], 1).astype(np.float32)
    n_ref, m_ref, _ = O.search_for_initialization(fa, fb, prev.reshape(-1), nnratio=0.9, check_ori=False)
    m = amd.ORBmatcher(0.9, False)
    n, m12 = m.SearchForInitialization(amd.Frame(a["kps"], a["desc"]), amd.Frame(b["kps"], b["desc"]), prev.copy(), 100)
    assert n == n_ref and np.array_equal(m12, m_ref)


def test_search_for_initialization_duplicate_descriptors(amd):
    """Identical descriptors everywhere: every tie is decided by candidate order and
    later F1 keypoints steal matches (R/src/ORBmatcher.cpp:538-566)."""
    rng = np.random.default_rng(5)
    n1 = 300
    from orb_slam2_amd import _abi
    k = np.zeros(n1, _abi.KEYPOINT_DTYPE)
    k["x"] = rng.integers(20, 620, n1)
    k["y"] = rng.integers(20, 460, n1)
    k["angle"] = rng.uniform(0, 360, n1).astype(np.float32)
    d = np.tile(rng.integers(0, 256, 32, dtype=np.uint8), (n1, 1))
    d[::3, 0] ^= 1
    prev = np.stack([k["x"], k["y"]], 1).astype(np.float32)
    fa = O.FrameView(k, d, 640, 480)
    n_ref, m_ref, p_ref = O.search_for_initialization(fa, fa, prev.reshape(-1), nnratio=1.01, window=40)
    m = amd.ORBmatcher(1.01, True)
    pg = prev.copy()
    n, m12 = m.SearchForInitialization(amd.Frame(k, d), amd.Frame(k, d), pg, 40)
    assert n == n_ref and np.array_equal(m12, m_ref) and np.array_equal(pg.reshape(-1), p_ref)


def _sbp_setup(W=640, H=480, nf=1000, seed=0x5EED0001, stereo=False):
    a, b = _pair(W, H, seed, nf)
    rng = np.random.default_rng(11)
    fx, fy, cx, cy = 517.306408, 516.469215, 318.643040, 255.313989
    mbf = 40.0
    cam = np.array([fx, fy, cx, cy, mbf, mbf / fx], np.float32)
    kl = a["kps"]
    n = len(kl)
    z = rng.uniform(2.5, 3.5, n).astype(np.float32)
    xyz = np.stack([(kl["x"] - cx) * z / fx, (kl["y"] - cy) * z / fy, z], 1).astype(np.float32)
    Tl = np.eye(4, dtype=np.float32)
    Tc = np.eye(4, dtype=np.float32)
    Tc[0, 3] = -2 * 3.0 / fx
    Tc[1, 3] = -1 * 3.0 / fy
    has = (rng.random(n) < 0.8).astype(np.int32)
    outl = (rng.random(n) < 0.05).astype(np.uint8)
    mpd = a["desc"].copy()
    flip = rng.integers(0, 32, n)
    mpd[np.arange(n), flip] ^= 0x11
    ur = None
    if stereo:
        ur = np.where(rng.random(len(b["kps"])) < 0.7, b["kps"]["x"] - mbf / 3.0, -1).astype(np.float32)
    sf = O.tables(O.params(nf))["scale"]
    return a, b, cam, xyz, Tl, Tc, has, outl, mpd, ur, sf


@pytest.mark.parametrize("stereo,th,temporal", [(False, 15.0, False), (True, 7.0, False), (True, 15.0, False),
                                                (True, 7.0, True), (True, 15.0, True), (False, 60.0, True),
                                                (False, 60.0, False)])
def test_search_by_projection_frame(amd, stereo, th, temporal):
    """temporal: 40 % of the last frame's map points have no observations (Tracking::UpdateLastFrame's
    temporal points, R/src/Tracking.cpp:1132-1137) and some current slots hold such a point on entry
    (-3): those slots stay candidates (R/src/ORBmatcher.cpp:1649-1651)."""
    a, b, cam, xyz, Tl, Tc, has, outl, mpd, ur, sf = _sbp_setup(stereo=stereo)
    cur = O.FrameView(b["kps"], b["desc"], 640, 480, uright=ur)
    last = O.FrameView(a["kps"], a["desc"], 640, 480)
    camo = O.Camera(*[float(v) for v in cam])
    init = np.full(len(b["kps"]), -1, np.int32)
    init[::17] = -2
    if temporal:
        rng = np.random.default_rng(12)
        has = np.where((has > 0) & (rng.random(len(has)) < 0.4), 2, has).astype(np.int32)
        init[5::19] = -3
    n_ref, mp_ref = O.search_by_projection_ff(cur, Tc[:3], last, Tl[:3], has, outl, xyz, mpd, sf, camo, th,
                                              not stereo, True, init)
    m = amd.ORBmatcher(0.9, True)
    C = amd.Frame(b["kps"], b["desc"], 640, 480, mvuRight=ur, mTcw=Tc, mvScaleFactors=sf)
    L = amd.Frame(a["kps"], a["desc"], 640, 480, mTcw=Tl, mvScaleFactors=sf)
    n, mp = m.SearchByProjection(C, L, th, not stereo, has, outl, xyz, mpd, cam, init)
    assert n == n_ref and np.array_equal(mp, mp_ref)
    assert n > 100


def test_knn2(amd):
    a, b = _pair(640, 480, 0x5EED0001, 1000)
    bi, bd, sd = O.hamming_knn2(a["desc"], b["desc"])
    m = amd.ORBmatcher()
    gi, gd, gs = m.knn2(a["desc"], b["desc"])
    assert np.array_equal(bi, gi) and np.array_equal(bd, gd) and np.array_equal(sd, gs)


def test_descriptor_distance(amd):
    rng = np.random.default_rng(2)
    for _ in range(50):
        x = rng.integers(0, 256, 32, dtype=np.uint8)
        y = rng.integers(0, 256, 32, dtype=np.uint8)
        assert amd.ORBmatcher.DescriptorDistance(x, y) == O.descriptor_distance(x, y)


def _sbl_setup(W=640, H=480, nf=1000, seed=0x5EED0001, stereo=False, n_mp=700, rs=21):
    """Local map points near the current frame's keypoints: projections within ~1 px of a
    keypoint (plus strays), descriptors with a few flipped bits, random levels around the
    keypoint octave, viewing cosines on both sides of 0.998, 10 % out of view, 5 % without
    observations; some slots of mvpMapPoints pre-occupied (with / without observations)."""
    from orb_slam2_amd import synth
    cv = synth.canvas(seed, W, H)
    p = O.params(nf)
    b = O.extract(p, synth.frame(cv, W, H, 1))
    rng = np.random.default_rng(rs)
    kc = b["kps"]
    src = rng.integers(0, len(kc), n_mp)
    proj = np.zeros((n_mp, 3), np.float32)
    proj[:, 0] = kc["x"][src] + rng.normal(0, 1.0, n_mp)
    proj[:, 1] = kc["y"][src] + rng.normal(0, 1.0, n_mp)
    stray = rng.random(n_mp) < 0.1
    proj[stray, 0] = rng.uniform(0, W, stray.sum())
    proj[stray, 1] = rng.uniform(0, H, stray.sum())
    level = np.clip(kc["octave"][src] + rng.integers(-1, 2, n_mp), 0, 7).astype(np.int32)
    view_cos = np.where(rng.random(n_mp) < 0.5, 0.999, 0.99).astype(np.float32)
    desc = b["desc"][src].copy()
    for _ in range(3):
        desc[np.arange(n_mp), rng.integers(0, 32, n_mp)] ^= (1 << rng.integers(0, 8, n_mp)).astype(np.uint8)
    in_view = rng.random(n_mp) > 0.1
    has_obs = rng.random(n_mp) > 0.05
    ur = None
    if stereo:
        ur = np.where(rng.random(len(kc)) < 0.7, kc["x"] - 12.0, -1).astype(np.float32)
        proj[:, 2] = proj[:, 0] - 12.0 + rng.normal(0, 2.0, n_mp)
    init = np.full(len(kc), -1, np.int32)
    init[::23] = -2
    init[5::31] = -3
    sf = O.tables(p)["scale"]
    return b, in_view, proj, level, view_cos, desc, has_obs, ur, init, sf


@pytest.mark.parametrize("stereo,th,nn", [(False, 3.0, 0.8), (True, 3.0, 0.8), (False, 1.0, 0.8), (True, 5.0, 0.6)])
def test_search_by_projection_local(amd, stereo, th, nn):
    b, in_view, proj, level, vcos, desc, has_obs, ur, init, sf = _sbl_setup(stereo=stereo)
    f = O.FrameView(b["kps"], b["desc"], 640, 480, uright=ur)
    n_ref, mp_ref = O.search_by_projection_local(f, in_view, proj, level, vcos, desc, has_obs, sf, nn, th, init)
    m = amd.ORBmatcher(nn, True)
    F = amd.Frame(b["kps"], b["desc"], 640, 480, mvuRight=ur, mvScaleFactors=sf)
    mp = amd.LocalMapPoints(in_view, proj, level, vcos, desc, has_obs)
    n, cur = m.SearchByProjectionLocal(F, mp, th, init)
    assert n == n_ref and np.array_equal(cur, mp_ref)
    assert n > 200
