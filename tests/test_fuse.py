"""ORBmatcher::Fuse (matching step): the oracle's behaviour on synthetic keyframes (CPU) and the
gfx950 kernel bit-exact against the oracle (GPU)."""
import numpy as np
import pytest

import oracle_ref as O


def _prob(**kw):
    from orb_slam2_amd import synth
    return synth.fuse_problem(**kw)


def test_fuse_oracle_finds_true_points():
    p = _prob()
    bi, bd = O.fuse(p)
    assert (bi >= 0).sum() > 0.3 * len(bi)
    assert np.all(bd[bi >= 0] <= 50)
    assert np.all(bi[p["mp_valid"] == 0] == -1)
    # a matched keypoint is within the search square and close in descriptor space
    kf = p["kf"]
    for i in np.nonzero(bi >= 0)[0][:50]:
        assert O.descriptor_distance(p["mp_desc"][i], kf["desc"][bi[i]]) == bd[i]


def _gpu(amd, p, th):
    from orb_slam2_amd import Frame
    import numpy as np
    kf = p["kf"]
    k = np.zeros(len(kf["x"]), dtype=[("x", "f4"), ("y", "f4"), ("size", "f4"), ("angle", "f4"), ("response", "f4"),
                                     ("octave", "i4"), ("class_id", "i4")])
    k["x"], k["y"], k["octave"] = kf["x"], kf["y"], kf["octave"]
    fr = Frame(k, kf["desc"], kf["W"], kf["H"], mvuRight=kf["uright"])
    kp = p["kp"]
    return amd.Fuse(fr, kp["Tcw"], kp["Ow"], kp["cam"], kp["log_scale_factor"], kp["scale_factors"],
                    kp["inv_level_sigma2"], p["mp_valid"], p["mp_xyz"], p["mp_normal"], p["mp_min_dist"],
                    p["mp_max_dist"], p["mp_desc"], th)


@pytest.mark.gpu
@pytest.mark.parametrize("kw,th", [(dict(), 3.0), (dict(seed=7, stereo_frac=0.0), 5.0),
                                   (dict(seed=11, n_kps=3000, n_mp=2000, true_frac=0.8), 3.0),
                                   (dict(seed=4, n_kps=5, n_mp=40), 3.0)])
def test_fuse_gpu_matches_oracle(amd, kw, th):
    p = _prob(**kw)
    bi, bd = O.fuse(p, th)
    gi, gd = _gpu(amd, p, th)
    assert np.array_equal(gi, bi)
    assert np.array_equal(gd, bd)


def _py_fuse(p, th=3.0):
    """Literal Python restatement of R/src/ORBmatcher.cpp:1006-1121 (float32 scalars, the same
    OpenCV-product restatements as the oracle), with GetFeaturesInArea of R/src/KeyFrame.cpp:702-743
    over the PosInGrid grid of R/src/Frame.cpp:442-452."""
    f32 = np.float32
    kf, kp = p["kf"], p["kp"]
    W, H = kf["W"], kf["H"]
    winv, hinv = f32(64) / f32(W), f32(48) / f32(H)
    grid = [[[] for _ in range(48)] for _ in range(64)]
    for i, (x, y) in enumerate(zip(kf["x"], kf["y"])):
        gx, gy = int(np.round(f32(x - f32(0)) * winv)), int(np.round(f32(y - f32(0)) * hinv))
        if 0 <= gx < 64 and 0 <= gy < 48:
            grid[gx][gy].append(i)
    T, Ow = np.asarray(kp["Tcw"], f32), np.asarray(kp["Ow"], f32)
    fx, fy, cx, cy, bf = (f32(v) for v in kp["cam"])
    sf, isg = kp["scale_factors"], kp["inv_level_sigma2"]
    out_i, out_d = [], []
    for i in range(len(p["mp_valid"])):
        bi, bd = -1, 256
        X = p["mp_xyz"][i]
        while p["mp_valid"][i]:
            p3 = [f32(float(T[r, 0]) * float(X[0]) + float(T[r, 1]) * float(X[1]) + float(T[r, 2]) * float(X[2])
                      + float(T[r, 3])) for r in range(3)]
            if p3[2] < f32(0):
                break
            invz = f32(1) / p3[2]
            u = fx * (p3[0] * invz) + cx
            v = fy * (p3[1] * invz) + cy
            if not (u >= 0 and u < W and v >= 0 and v < H):
                break
            ur = u - bf * invz
            PO = [X[k] - Ow[k] for k in range(3)]
            dist = f32(np.sqrt(float((PO[0] * PO[0] + PO[1] * PO[1]) + PO[2] * PO[2])))
            if dist < f32(0.8) * p["mp_min_dist"][i] or dist > f32(1.2) * p["mp_max_dist"][i]:
                break
            Pn = p["mp_normal"][i]
            if float((PO[0] * Pn[0] + PO[1] * Pn[1]) + PO[2] * Pn[2]) < 0.5 * float(dist):
                break
            lev = int(np.ceil(np.log(float(p["mp_max_dist"][i] / dist)) / float(f32(kp["log_scale_factor"]))))
            lev = min(max(lev, 0), kp["n_levels"] - 1)
            r = f32(th) * sf[lev]
            x0 = max(0, int(np.floor(f32(u - f32(0) - r) * winv)))
            x1 = min(63, int(np.ceil(f32(u - f32(0) + r) * winv)))
            y0 = max(0, int(np.floor(f32(v - f32(0) - r) * hinv)))
            y1 = min(47, int(np.ceil(f32(v - f32(0) + r) * hinv)))
            if x0 >= 64 or x1 < 0 or y0 >= 48 or y1 < 0:
                break
            for ix in range(x0, x1 + 1):
                for iy in range(y0, y1 + 1):
                    for j in grid[ix][iy]:
                        if not (abs(kf["x"][j] - u) < r and abs(kf["y"][j] - v) < r):
                            continue
                        lv = kf["octave"][j]
                        if lv < lev - 1 or lv > lev:
                            continue
                        ex, ey = u - kf["x"][j], v - kf["y"][j]
                        if kf["uright"][j] >= 0:
                            er = ur - kf["uright"][j]
                            if float((ex * ex + ey * ey + er * er) * isg[lv]) > 7.8:
                                continue
                        elif float((ex * ex + ey * ey) * isg[lv]) > 5.99:
                            continue
                        d = O.descriptor_distance(p["mp_desc"][i], kf["desc"][j])
                        if d < bd:
                            bd, bi = d, j
            break
        out_i.append(bi if bd <= 50 else -1)
        out_d.append(bd)
    return np.array(out_i, np.int32), np.array(out_d, np.int32)


def test_fuse_oracle_vs_python_restatement():
    p = _prob(seed=9, n_kps=400, n_mp=150)
    bi, bd = O.fuse(p)
    pi, pd = _py_fuse(p)
    assert np.array_equal(bi, pi) and np.array_equal(bd, pd)


def test_fuse_sim3_oracle_drops_only_the_reprojection_gate():
    """The Scw form (R/src/ORBmatcher.cpp:1164-1261) keeps every Fuse gate but the reprojection
    test, so it matches at least the points Fuse matches at the same radius."""
    p = _prob(seed=5)
    bi, _ = O.fuse(p, 4.0)
    si, _ = O.fuse(p, 4.0, sim3=True)
    assert np.all(si[bi >= 0] >= 0) and (si >= 0).sum() >= (bi >= 0).sum()


@pytest.mark.gpu
@pytest.mark.parametrize("kw,th", [(dict(), 4.0), (dict(seed=9, n_kps=3000, n_mp=2000, true_frac=0.8), 4.0),
                                   (dict(seed=13, stereo_frac=0.5), 8.0)])
def test_fuse_sim3_gpu_matches_oracle(amd, kw, th):
    from orb_slam2_amd import Frame
    p = _prob(**kw)
    bi, bd = O.fuse(p, th, sim3=True)
    kf, kp = p["kf"], p["kp"]
    k = np.zeros(len(kf["x"]), dtype=[("x", "f4"), ("y", "f4"), ("size", "f4"), ("angle", "f4"), ("response", "f4"),
                                     ("octave", "i4"), ("class_id", "i4")])
    k["x"], k["y"], k["octave"] = kf["x"], kf["y"], kf["octave"]
    fr = Frame(k, kf["desc"], kf["W"], kf["H"])
    gi, gd = amd.FuseSim3(fr, kp["Tcw"], kp["Ow"], kp["cam"], kp["log_scale_factor"], kp["scale_factors"],
                          p["mp_valid"], p["mp_xyz"], p["mp_normal"], p["mp_min_dist"], p["mp_max_dist"], p["mp_desc"],
                          th)
    assert np.array_equal(gi, bi) and np.array_equal(gd, bd)
