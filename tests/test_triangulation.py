"""ORBmatcher::SearchForTriangulation: the oracle against a literal Python restatement of the
reference loop (CPU), and the gfx950 kernels bit-exact against the oracle (GPU)."""
import numpy as np
import pytest

import oracle_ref as O


def _prob(**kw):
    from orb_slam2_amd import synth
    return synth.triangulation_problem(**kw)


def _py(p, only_stereo=False, check_ori=True):
    """R/src/ORBmatcher.cpp:785-983 with CheckDistEpipolarLine (:175-203), float32 scalars."""
    f32 = np.float32
    k1, k2, F = p["kf1"], p["kf2"], p["F12"]
    ex, ey = f32(p["ex"]), f32(p["ey"])
    fv1 = {int(n): list(k1["fidx"][k1["start"][i]:k1["start"][i + 1]]) for i, n in enumerate(k1["nodes"])}
    fv2 = {int(n): list(k2["fidx"][k2["start"][i]:k2["start"][i + 1]]) for i, n in enumerate(k2["nodes"])}
    matched2 = np.zeros(len(k2["x"]), bool)
    m12 = -np.ones(len(k1["x"]), np.int32)
    for node in sorted(set(fv1) & set(fv2)):
        for i1 in fv1[node]:
            if k1["has_mp"][i1]:
                continue
            st1 = k1["uright"][i1] >= 0
            if only_stereo and not st1:
                continue
            best, bi = 50, -1
            for i2 in fv2[node]:
                if matched2[i2] or k2["has_mp"][i2]:
                    continue
                st2 = k2["uright"][i2] >= 0
                if only_stereo and not st2:
                    continue
                d = O.descriptor_distance(k1["desc"][i1], k2["desc"][i2])
                if d > 50 or d > best:
                    continue
                x2, y2 = k2["x"][i2], k2["y"][i2]
                if not st1 and not st2:
                    dx, dy = ex - x2, ey - y2
                    if dx * dx + dy * dy < f32(100) * p["scale_factors"][k2["octave"][i2]]:
                        continue
                x1, y1 = k1["x"][i1], k1["y"][i1]
                a = x1 * F[0, 0] + y1 * F[1, 0] + F[2, 0]
                b = x1 * F[0, 1] + y1 * F[1, 1] + F[2, 1]
                c = x1 * F[0, 2] + y1 * F[1, 2] + F[2, 2]
                num, den = a * x2 + b * y2 + c, a * a + b * b
                if den == 0 or not float(num * num / den) < 3.84 * float(p["level_sigma2"][k2["octave"][i2]]):
                    continue
                best, bi = d, i2
            if bi >= 0:
                m12[i1] = bi
                matched2[bi] = True
    if check_ori:
        def rbin(i):
            rot = k1["angle"][i] - k2["angle"][m12[i]]
            if rot < 0.0:
                rot += f32(360.0)
            b = int(np.floor(float(rot * (f32(30) / f32(360.0))) + 0.5))   # roundf (half away from zero, rot >= 0)
            return 0 if b == 30 else b
        hist = np.zeros(30, int)
        for i in np.nonzero(m12 >= 0)[0]:
            hist[rbin(i)] += 1
        order = []
        m1 = m2 = m3 = 0
        i1 = i2 = i3 = -1
        for i, s in enumerate(hist):
            if s > m1:
                m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
            elif s > m2:
                m3, m2, i3, i2 = m2, s, i2, i
            elif s > m3:
                m3, i3 = s, i
        if f32(m2) < f32(0.1) * f32(m1):
            i2 = i3 = -1
        elif f32(m3) < f32(0.1) * f32(m1):
            i3 = -1
        for i in np.nonzero(m12 >= 0)[0]:
            if rbin(i) not in (i1, i2, i3):
                m12[i] = -1
        del order
    return int((m12 >= 0).sum()), m12


@pytest.mark.parametrize("only_stereo,check_ori", [(False, True), (False, False), (True, True)])
def test_oracle_vs_python(only_stereo, check_ori):
    p = _prob(seed=5, n_points=300, extra=60, n_nodes=400)
    n, m = O.search_for_triangulation(p, only_stereo, check_ori)
    pn, pm = _py(p, only_stereo, check_ori)
    assert n == pn and np.array_equal(m, pm)
    if not only_stereo:
        assert n > 30


def _frame(k):
    from orb_slam2_amd import Frame
    kp = np.zeros(len(k["x"]), dtype=[("x", "f4"), ("y", "f4"), ("size", "f4"), ("angle", "f4"), ("response", "f4"),
                                      ("octave", "i4"), ("class_id", "i4")])
    kp["x"], kp["y"], kp["angle"], kp["octave"] = k["x"], k["y"], k["angle"], k["octave"]
    return Frame(kp, k["desc"], k["W"], k["H"], mvuRight=k["uright"])


@pytest.mark.gpu
@pytest.mark.parametrize("kw,only_stereo,check_ori", [
    (dict(), False, True), (dict(seed=8), False, False), (dict(seed=9, stereo_frac=0.6), True, True),
    (dict(seed=10, n_points=3000, extra=500, n_nodes=200), False, True),   # crowded nodes
])
def test_search_for_triangulation_gpu(amd, kw, only_stereo, check_ori):
    p = _prob(**kw)
    n, m = O.search_for_triangulation(p, only_stereo, check_ori)
    k1, k2 = p["kf1"], p["kf2"]
    gn, gm = amd.SearchForTriangulation(_frame(k1), _frame(k2), k1["has_mp"], k2["has_mp"],
                                        (k1["nodes"], k1["start"], k1["fidx"]), (k2["nodes"], k2["start"], k2["fidx"]),
                                        p["F12"], (p["ex"], p["ey"]), p["scale_factors"], p["level_sigma2"],
                                        only_stereo, check_ori)
    assert gn == n and np.array_equal(gm, m)
