"""CPU-only checks of the oracle: known-answer constants of the reference,
cross-checks against independent numpy / pure-Python restatements, and the
glibc sinf/cosf pin."""
import hashlib
import math
import os
import pathlib

import numpy as np
import pytest

import oracle_ref as O
import pyref_octree

ROOT = pathlib.Path(__file__).resolve().parents[1]


# ---------------------------------------------------------------- A1 constants

def test_umax_table():
    assert O.tables(O.params())["umax"].tolist() == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]


@pytest.mark.parametrize("nf,quota", [
    (1000, [217, 181, 151, 126, 105, 87, 73, 60]),
    (2000, [434, 362, 302, 251, 209, 175, 145, 122]),
    (1200, [261, 217, 181, 151, 126, 105, 87, 72]),
])
def test_features_per_level(nf, quota):
    fpl = O.tables(O.params(nf))["features_per_level"]
    assert fpl.tolist() == quota and fpl.sum() == nf


def test_scale_factors_and_sizes():
    t = O.tables(O.params())
    assert np.allclose(t["scale"], [1, 1.2, 1.44, 1.728, 2.0736, 2.48832, 2.985985, 3.583182], rtol=1e-6)
    assert [int(np.float32(31) * s) for s in t["scale"]] == [31, 37, 44, 53, 64, 77, 92, 111]
    lw, lh = O.level_sizes(O.params(), 640, 480)
    assert list(zip(lw, lh)) == [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231), (257, 193),
                                 (214, 161), (179, 134)]
    lw, lh = O.level_sizes(O.params(2000), 1241, 376)
    assert list(zip(lw, lh)) == [(1241, 376), (1034, 313), (862, 261), (718, 218), (598, 181), (499, 151),
                                 (416, 126), (346, 105)]


def test_pattern_table():
    txt = (ROOT / "orb-slam2-_amd" / "csrc" / "orb_pattern.inc").read_text().split("\n", 1)[1]
    vals = [int(v) for v in txt.replace(",", " ").split()]
    assert len(vals) == 1024 and min(vals) == -13 and max(vals) == 12
    assert vals[:8] == [8, -3, 9, 5, 4, 2, 7, -12]
    assert hashlib.sha256(np.array(vals, np.int8).tobytes()).hexdigest() == "2164181aea6ff9ac426ca512d5130d15e1f6e3cd47b1cbdd568bbe1e55d49023"


# ---------------------------------------------------------------- A2/A6 primitives vs numpy

def test_resize_constant_and_numpy():
    rng = np.random.default_rng(0)
    src = rng.integers(0, 256, (97, 131), dtype=np.uint8)
    dh, dw = 81, 109
    got = O.resize(src, dw, dh)
    # independent numpy restatement of the fixed-point INTER_LINEAR path
    def coeffs(d, s, clamp):
        sc = 1.0 / (d / s)
        f = ((np.arange(d) + 0.5) * sc - 0.5).astype(np.float32)
        i = np.floor(f).astype(np.int64)
        f = (f - i.astype(np.float32)).astype(np.float32)
        if clamp:
            f = np.where(i < 0, np.float32(0), f); i = np.maximum(i, 0)
            f = np.where(i >= s - 1, np.float32(0), f); i = np.minimum(i, s - 1)
        a0 = np.rint((np.float32(1) - f) * np.float32(2048)).astype(np.int64)
        a1 = np.rint(f * np.float32(2048)).astype(np.int64)
        return i, a0, a1
    xi, xa0, xa1 = coeffs(dw, 131, True)
    yi, yb0, yb1 = coeffs(dh, 97, False)
    S = src.astype(np.int64)
    x1 = np.minimum(xi + 1, 130)
    rows = S[:, xi] * xa0 + S[:, x1] * xa1
    y0 = np.clip(yi, 0, 96); y1 = np.clip(yi + 1, 0, 96)
    ref = (rows[y0] * yb0[:, None] + rows[y1] * yb1[:, None] + (1 << 21)) >> 22
    assert np.array_equal(got, np.clip(ref, 0, 255).astype(np.uint8))
    assert np.all(O.resize(np.full((480, 640), 77, np.uint8), 533, 400) == 77)


def test_blur_kernel_sum_257_artifact():
    """getGaussianKernel(7,2) rounded to 8 bits sums to 257: a flat 100 blurs to 101."""
    assert np.all(O.blur(np.full((40, 50), 100, np.uint8)) == 101)
    assert np.all(O.blur(np.full((40, 50), 255, np.uint8)) == 255)


# ---------------------------------------------------------------- A3 FAST

def test_fast_single_corner():
    img = np.full((40, 40), 100, np.uint8)
    img[21, 17] = 200            # an isolated bright pixel: all 16 ring pixels darker by 100
    kps = O.fast_roi(img, 0, 0, 40, 40, 20)
    assert kps.tolist() == [[17, 21, 99]]
    img[21, 17] = 100
    img[20:, 20:] = 200          # a right-angle corner: equal scores along the edge suppress each other
    assert O.fast_roi(img, 0, 0, 40, 40, 20).size == 0
    assert O.fast_roi(np.full((40, 40), 9, np.uint8), 0, 0, 40, 40, 7).size == 0


def test_fast_threshold_monotone():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (64, 64), dtype=np.uint8)
    lo = {(x, y) for x, y, s in O.fast_roi(img, 0, 0, 64, 64, 7)}
    hi = {(x, y, s) for x, y, s in O.fast_roi(img, 0, 0, 64, 64, 40)}
    assert all(s >= 40 for _, _, s in hi)
    assert len(lo) > 0


# ---------------------------------------------------------------- A5 fastAtan2

def test_fast_atan2_known_values():
    assert O.fast_atan2(0.0, 1.0) == 0.0
    assert abs(O.fast_atan2(1.0, 0.0) - 90.0) < 1e-3
    assert abs(O.fast_atan2(0.0, -1.0) - 180.0) < 1e-3
    assert abs(O.fast_atan2(-1.0, 0.0) - 270.0) < 1e-3
    rng = np.random.default_rng(4)
    for y, x in rng.integers(-100000, 100000, (200, 2)):
        ref = math.degrees(math.atan2(y, x)) % 360
        got = O.fast_atan2(float(y), float(x))
        assert min(abs(got - ref), 360 - abs(got - ref)) < 0.02   # OpenCV's polynomial is ~0.01 deg


# ---------------------------------------------------------------- N3 sinf/cosf

def test_sincosf_matches_host_libm():
    """The restated glibc sinf/cosf equals the host libm bit for bit (the FMA ifunc variant).
    Default: every 61st float in [0, 2pi]; ORB_SINCOS_EXHAUSTIVE=1 checks all 1.09e9."""
    import ctypes as C
    f = O.lib().oracle_sincosf_check
    f.restype = C.c_long
    f.argtypes = [C.c_uint, C.POINTER(C.c_long)]
    n = C.c_long()
    stride = 1 if os.environ.get("ORB_SINCOS_EXHAUSTIVE") == "1" else 61
    bad = f(stride, C.byref(n))
    assert n.value > 17_000_000 // stride * 1 or stride == 1
    assert bad == 0, f"{bad} of {n.value} inputs differ from libm"


# ---------------------------------------------------------------- A4 octree vs pure Python

@pytest.mark.parametrize("seed,n,N", [(0, 50, 10), (1, 300, 37), (2, 800, 120), (3, 2000, 217), (4, 40, 100),
                                      (5, 500, 1), (6, 0, 10)])
def test_octree_matches_python_list_restatement(seed, n, N):
    rng = np.random.default_rng(seed)
    W, H = 608, 448
    kx = rng.integers(3, W - 4, n).astype(np.float32)
    ky = rng.integers(3, H - 4, n).astype(np.float32)
    if n > 10:       # duplicate coordinates (overlapping FAST cells) and clusters
        kx[: n // 10] = kx[n // 10: 2 * (n // 10)]
        ky[: n // 10] = ky[n // 10: 2 * (n // 10)]
    kr = rng.integers(7, 120, n).astype(np.float32)
    got = O.distribute_octree(kx, ky, kr, 16, 16 + W, 16, 16 + H, N) if n else []
    ref = pyref_octree.distribute_octree(kx, ky, kr, 16, 16 + W, 16, 16 + H, N) if n else []
    assert list(got) == ref


# ---------------------------------------------------------------- A9 Hamming

def test_descriptor_distance_popcount():
    rng = np.random.default_rng(9)
    for _ in range(100):
        a = rng.integers(0, 256, 32, dtype=np.uint8)
        b = rng.integers(0, 256, 32, dtype=np.uint8)
        assert O.descriptor_distance(a, b) == int(np.unpackbits(a ^ b).sum())
    assert O.descriptor_distance(np.zeros(32, np.uint8), np.full(32, 255, np.uint8)) == 256


def _py_features_in_area(kx, ky, oct_, W, H, x, y, r, minL, maxL):
    """Frame::AssignFeaturesToGrid + GetFeaturesInArea restated in Python (R/src/Frame.cpp:244-260, 387-452)."""
    winv, hinv = np.float32(64) / np.float32(W), np.float32(48) / np.float32(H)
    grid = [[[] for _ in range(48)] for _ in range(64)]
    for i in range(len(kx)):
        px = int(np.round(np.float32(kx[i]) * winv))
        py = int(np.round(np.float32(ky[i]) * hinv))
        if 0 <= px < 64 and 0 <= py < 48:
            grid[px][py].append(i)
    x, y, r = np.float32(x), np.float32(y), np.float32(r)
    cx0 = max(0, int(np.floor((x - r) * winv)))
    if cx0 >= 64:
        return []
    cx1 = min(63, int(np.ceil((x + r) * winv)))
    if cx1 < 0:
        return []
    cy0 = max(0, int(np.floor((y - r) * hinv)))
    if cy0 >= 48:
        return []
    cy1 = min(47, int(np.ceil((y + r) * hinv)))
    if cy1 < 0:
        return []
    check = minL > 0 or maxL >= 0
    out = []
    for ix in range(cx0, cx1 + 1):
        for iy in range(cy0, cy1 + 1):
            for i in grid[ix][iy]:
                if check:
                    if oct_[i] < minL:
                        continue
                    if maxL >= 0 and oct_[i] > maxL:
                        continue
                if abs(np.float32(kx[i]) - x) < r and abs(np.float32(ky[i]) - y) < r:
                    out.append(i)
    return out


def test_search_by_projection_local_oracle_vs_python():
    """The C oracle of SearchByProjection(Frame&, vector<MapPoint*>, th) against a literal
    Python restatement of R/src/ORBmatcher.cpp:63-163 on a small random frame."""
    rng = np.random.default_rng(3)
    n, n_mp = 260, 220
    from orb_slam2_amd import _abi
    k = np.zeros(n, _abi.KEYPOINT_DTYPE)
    k["x"] = rng.uniform(20, 620, n).astype(np.float32)
    k["y"] = rng.uniform(20, 460, n).astype(np.float32)
    k["octave"] = rng.integers(0, 4, n)
    d = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    ur = np.where(rng.random(n) < 0.5, k["x"] - 10, -1).astype(np.float32)
    src = rng.integers(0, n, n_mp)
    proj = np.stack([k["x"][src] + rng.normal(0, 2, n_mp), k["y"][src] + rng.normal(0, 2, n_mp),
                     k["x"][src] - 10 + rng.normal(0, 3, n_mp)], 1).astype(np.float32)
    level = np.clip(k["octave"][src] + rng.integers(-1, 2, n_mp), 0, 3).astype(np.int32)
    vcos = np.where(rng.random(n_mp) < 0.5, 0.999, 0.9).astype(np.float32)
    md = d[src].copy()
    md[np.arange(n_mp), rng.integers(0, 32, n_mp)] ^= 0x0F
    md[rng.random(n_mp) < 0.3] = d[rng.integers(0, n, 1)]    # many near-ties
    in_view = rng.random(n_mp) > 0.1
    has_obs = rng.random(n_mp) > 0.2
    sf = (np.float32(1.2) ** np.arange(8)).astype(np.float32)
    init = np.full(n, -1, np.int32)
    init[::13] = -2
    init[4::17] = -3
    th, nn = 2.0, 0.8
    f = O.FrameView(k, d, 640, 480, uright=ur)
    n_c, mp_c = O.search_by_projection_local(f, in_view, proj, level, vcos, md, has_obs, sf, nn, th, init)
    cur = init.copy()
    nm = 0
    pop = lambda a: bin(int(a)).count("1")
    for i in range(n_mp):
        if not in_view[i]:
            continue
        L = int(level[i])
        r = np.float32(2.5) if vcos[i] > np.float32(0.998) else np.float32(4.0)
        r = np.float32(r * np.float32(th))
        rad = np.float32(r * sf[L])
        cand = _py_features_in_area(k["x"], k["y"], k["octave"], 640, 480, proj[i, 0], proj[i, 1], rad, L - 1, L)
        bd, bl, bd2, bl2, bi = 256, -1, 256, -1, -1
        for idx in cand:
            s = cur[idx]
            if s == -2 or (s >= 0 and has_obs[s]):
                continue
            if ur[idx] > 0 and abs(np.float32(proj[i, 2]) - ur[idx]) > rad:
                continue
            dist = sum(pop(a ^ b) for a, b in zip(md[i], d[idx]))
            if dist < bd:
                bd2, bl2, bd, bl, bi = bd, bl, dist, int(k["octave"][idx]), idx
            elif dist < bd2:
                bl2, bd2 = int(k["octave"][idx]), dist
        if bd <= 100:
            if bl == bl2 and np.float32(bd) > np.float32(nn) * np.float32(bd2):
                continue
            cur[bi] = i
            nm += 1
    assert nm == n_c and np.array_equal(cur, mp_c)
    assert nm > 30


def test_search_by_projection_frame_oracle_vs_python():
    """The C oracle of SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
    against a literal Python restatement of R/src/ORBmatcher.cpp:1564-1718, with the last frame's
    map points as objects that do or do not have observations (Tracking::UpdateLastFrame's temporal
    points have none, R/src/Tracking.cpp:1132-1137) and current slots pre-set to points with and
    without observations: a slot whose point has no observations stays a candidate, so a later last
    point can take it over, and the rotation histogram then lists the slot twice."""
    from orb_slam2_amd import _abi
    rng = np.random.default_rng(5)
    W, H, n, nl = 640, 480, 300, 260
    kc = np.zeros(n, _abi.KEYPOINT_DTYPE)
    kc["x"] = rng.uniform(20, 620, n).astype(np.float32)
    kc["y"] = rng.uniform(20, 460, n).astype(np.float32)
    kc["octave"] = rng.integers(0, 3, n)
    kc["angle"] = rng.uniform(0, 360, n).astype(np.float32)
    dc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    urc = np.where(rng.random(n) < 0.5, kc["x"] - 12, -1).astype(np.float32)
    src = rng.integers(0, n, nl)                       # last keypoints near current ones (crowded)
    kl = np.zeros(nl, _abi.KEYPOINT_DTYPE)
    kl["x"] = (kc["x"][src] + rng.normal(0, 1.5, nl)).astype(np.float32)
    kl["y"] = (kc["y"][src] + rng.normal(0, 1.5, nl)).astype(np.float32)
    kl["octave"] = np.clip(kc["octave"][src] + rng.integers(-1, 2, nl), 0, 2)
    kl["angle"] = np.where(rng.random(nl) < 0.8, kc["angle"][src] + rng.normal(0, 3, nl),
                           rng.uniform(0, 360, nl)).astype(np.float32) % np.float32(360)
    dl = rng.integers(0, 256, (nl, 32), dtype=np.uint8)
    fx, fy, cx, cy, mbf = 500.0, 500.0, 320.0, 240.0, 40.0
    cam = np.array([fx, fy, cx, cy, mbf, mbf / fx], np.float32)
    z = rng.uniform(2.0, 4.0, nl).astype(np.float32)
    xyz = np.stack([(kl["x"] - cx) * z / fx, (kl["y"] - cy) * z / fy, z], 1).astype(np.float32)
    md = dc[src].copy()
    md[np.arange(nl), rng.integers(0, 32, nl)] ^= 0x07
    md[rng.random(nl) < 0.2] = dc[rng.integers(0, n)]          # near-ties
    has = rng.choice([0, 1, 2], nl, p=[0.15, 0.45, 0.4]).astype(np.int32)
    outl = (rng.random(nl) < 0.05).astype(np.uint8)
    Tl = np.eye(4, dtype=np.float32)[:3].copy()
    Tc = np.eye(4, dtype=np.float32)[:3].copy()
    Tc[0, 3], Tc[2, 3] = np.float32(0.004), np.float32(0.02)
    sf = (np.float32(1.2) ** np.arange(8)).astype(np.float32)
    init = np.full(n, -1, np.int32)
    init[::11] = -2
    init[5::13] = -3
    cur = O.FrameView(kc, dc, W, H, uright=urc)
    last = O.FrameView(kl, dl, W, H)
    retaken = 0
    for th, mono in ((7.0, False), (15.0, True)):
        n_c, mp_c = O.search_by_projection_ff(cur, Tc, last, Tl, has, outl, xyz, md, sf, O.Camera(*map(float, cam)),
                                              th, mono, True, init)
        # ---- literal restatement: slots hold ("pre", has_obs) or ("last", i)
        slot = [None if v == -1 else ("pre", v == -2) for v in init]
        obs = lambda s: s[1] if s[0] == "pre" else has[s[1]] == 1
        f32 = np.float32
        twc = [f32(-sum(float(Tc[r, c]) * float(Tc[r, 3]) for r in range(3))) for c in range(3)]
        tlc2 = f32(sum(float(Tl[2, c]) * float(twc[c]) for c in range(3)) + float(Tl[2, 3]))
        bF = tlc2 > cam[5] and not mono
        bB = -tlc2 > cam[5] and not mono
        hist = [[] for _ in range(30)]
        nm = 0
        pop = lambda a: bin(int(a)).count("1")
        for i in range(nl):
            if not has[i] or outl[i]:
                continue
            x3 = [f32(sum(float(Tc[r, c]) * float(xyz[i, c]) for c in range(3)) + float(Tc[r, 3])) for r in range(3)]
            invz = f32(1.0 / float(x3[2]))
            if invz < 0:
                continue
            u = f32(f32(f32(cam[0] * x3[0]) * invz) + cam[2])
            v = f32(f32(f32(cam[1] * x3[1]) * invz) + cam[3])
            if u < 0 or u > W or v < 0 or v > H:
                continue
            lo = int(kl["octave"][i])
            rad = f32(f32(th) * sf[lo])
            if bF:
                cand = _py_features_in_area(kc["x"], kc["y"], kc["octave"], W, H, u, v, rad, lo, -1)
            elif bB:
                cand = _py_features_in_area(kc["x"], kc["y"], kc["octave"], W, H, u, v, rad, 0, lo)
            else:
                cand = _py_features_in_area(kc["x"], kc["y"], kc["octave"], W, H, u, v, rad, lo - 1, lo + 1)
            if not cand:
                continue
            bd, bi = 256, -1
            for i2 in cand:
                if slot[i2] is not None and obs(slot[i2]):
                    continue
                if urc[i2] > 0:
                    urp = f32(u - f32(cam[4] * invz))
                    if abs(f32(urp - urc[i2])) > rad:
                        continue
                dist = sum(pop(a ^ b) for a, b in zip(md[i], dc[i2]))
                if dist < bd:
                    bd, bi = dist, i2
            if bd <= 100:
                slot[bi] = ("last", i)
                nm += 1
                rot = f32(kl["angle"][i] - kc["angle"][bi])
                if rot < 0:
                    rot = f32(rot + f32(360))
                b = int(np.round(f32(rot * f32(f32(30) / f32(360)))))
                hist[0 if b == 30 else b].append(bi)
        sizes = [len(h) for h in hist]
        m1 = m2 = m3 = 0
        i1 = i2_ = i3 = -1
        for b, c in enumerate(sizes):
            if c > m1:
                m3, m2, m1, i3, i2_, i1 = m2, m1, c, i2_, i1, b
            elif c > m2:
                m3, m2, i3, i2_ = m2, c, i2_, b
            elif c > m3:
                m3, i3 = c, b
        if f32(m2) < f32(0.1) * f32(m1):
            i2_ = i3 = -1
        elif f32(m3) < f32(0.1) * f32(m1):
            i3 = -1
        for b in range(30):
            if b not in (i1, i2_, i3):
                for j in hist[b]:
                    slot[j] = None
                    nm -= 1
        want = np.array([-1 if s is None else (s[1] if s[0] == "last" else (-2 if s[1] else -3)) for s in slot], np.int32)
        assert nm == n_c and np.array_equal(want, mp_c), th
        assert nm > 20
        listed = [j for h in hist for j in h]
        retaken += len(listed) - len(set(listed))     # slots taken over from a point without observations
    assert retaken > 0


def test_compute_stereo_matches_oracle_vs_python():
    """The C oracle of Frame::ComputeStereoMatches against a literal Python restatement of
    R/src/Frame.cpp:551-770 (with mb = 0 at call time) on a synthetic stereo pair."""
    from orb_slam2_amd import synth
    W, H = 752, 480
    cv = synth.canvas(0x5EED0005, W, H)
    left, right = synth.stereo_pair(cv, W, H, 0)
    p = O.params(1200)
    a = O.extract(p, left, want_pyramid=True)
    b = O.extract(p, right, want_pyramid=True)
    mbf = float(np.float32(synth.CAMERAS["EUROC"]["bf"]))   # R/Examples/Stereo/EuRoC.yaml:25
    n_c, ur_c, dep_c = O.compute_stereo_matches(p, a, b, mbf)
    t = O.tables(p)
    lw, lh = a["sizes"]
    offs = np.concatenate([[0], np.cumsum(np.asarray(lw, np.int64) * lh)])
    lev = lambda pyr, l: pyr[offs[l]:offs[l + 1]].reshape(lh[l], lw[l]).astype(np.int64)
    kl, kr = a["kps"], b["kps"]
    popc = np.array([bin(i).count("1") for i in range(256)])
    rows = [[] for _ in range(lh[0])]
    for iR in range(len(kr)):
        r = np.float32(2.0) * t["scale"][kr["octave"][iR]]
        for yi in range(int(np.floor(kr["y"][iR] - r)), int(np.ceil(kr["y"][iR] + r)) + 1):
            rows[yi].append(iR)
    maxD = np.float32(np.inf)
    ur = np.full(len(kl), -1.0, np.float32)
    dep = np.full(len(kl), -1.0, np.float32)
    vd = []
    for iL in range(len(kl)):
        lv, uL, vL = int(kl["octave"][iL]), np.float32(kl["x"][iL]), np.float32(kl["y"][iL])
        cands = rows[int(vL)]
        if not cands:
            continue
        best, bi = 100, 0
        for iR in cands:
            if kr["octave"][iR] < lv - 1 or kr["octave"][iR] > lv + 1:
                continue
            if kr["x"][iR] <= uL:
                dist = int(popc[a["desc"][iL] ^ b["desc"][iR]].sum())
                if dist < best:
                    best, bi = dist, iR
        if best >= 75:
            continue
        sf = t["inv_scale"][lv]
        rnd = lambda v: np.float32(np.sign(v) * np.floor(np.abs(v) + np.float32(0.5)))   # round(): half away
        cx, cy, cr = int(rnd(np.float32(uL * sf))), int(rnd(np.float32(vL * sf))), int(rnd(np.float32(kr["x"][bi] * sf)))
        if cr < 0 or cr + 11 >= lw[lv]:
            continue
        IL, IR = lev(a["pyramid"], lv), lev(b["pyramid"], lv)
        wl = IL[cy - 5:cy + 6, cx - 5:cx + 6] - IL[cy, cx]
        dists = []
        for inc in range(-5, 6):
            wr = IR[cy - 5:cy + 6, cr + inc - 5:cr + inc + 6] - IR[cy, cr + inc]
            dists.append(float(np.abs(wl - wr).sum()))
        bs = int(np.argmin(dists))
        binc = bs - 5
        if binc in (-5, 5):
            continue
        d1, d2, d3 = (np.float32(dists[bs - 1]), np.float32(dists[bs]), np.float32(dists[bs + 1]))
        with np.errstate(divide="ignore", invalid="ignore"):
            delta = np.float32((d1 - d3) / (np.float32(2.0) * (d1 + d3 - np.float32(2.0) * d2)))
        if not (-1 <= delta <= 1):
            continue
        bu = np.float32(t["scale"][lv] * np.float32(np.float32(np.float32(cr) + np.float32(binc)) + delta))
        disp = np.float32(uL - bu)
        if disp >= 0 and disp < maxD:
            if disp <= 0:
                disp, bu = np.float32(0.01), np.float32(np.float64(uL) - 0.01)
            dep[iL] = np.float32(np.float32(mbf) / disp)
            ur[iL] = bu
            vd.append((int(dists[bs]), iL))
    vd.sort()
    if vd:
        th = np.float32(np.float32(1.5) * np.float32(1.4)) * np.float32(vd[len(vd) // 2][0])
        for dist, iL in reversed(vd):
            if np.float32(dist) < th:
                break
            ur[iL] = -1
            dep[iL] = -1
    assert np.array_equal(ur, ur_c) and np.array_equal(dep, dep_c)
    assert n_c == int((ur >= 0).sum()) and n_c > 300
