"""ORBmatcher::SearchByBoW, both overloads (R/src/ORBmatcher.cpp:220-372 keyframe-frame, :632-760
keyframe-keyframe): the C oracle against a literal Python restatement of the reference loops
(CPU), and the gfx950 one-wave-per-node kernel bit-exact against the oracle (GPU).  Inputs:
synth.bow_match_problem over a synthetic vocabulary, feature vectors from the oracle's
TemplatedVocabulary::transform.  Parity anchor: the reference ships no SearchByBoW fixtures; the
oracle is pinned by the restatement below."""
import numpy as np
import pytest

import oracle_ref as O

L = 4


def _problem(levelsup, seed=9, **kw):
    from orb_slam2_amd import synth
    voc = synth.vocabulary(k=8, L=L, seed=5, early_leaf=0.05, stop_frac=0.03)
    ov = O.OracleVocabulary(*voc, L)
    k1, k2 = synth.bow_match_problem(voc, seed=seed, **kw)
    fv1 = O.bow_transform(ov, k1["desc"], levelsup)[1]
    fv2 = O.bow_transform(ov, k2["desc"], levelsup)[1]
    return k1, k2, fv1, fv2


def _table(d1, d2):
    b1 = np.unpackbits(d1, axis=1).astype(np.int16)
    b2 = np.unpackbits(d2, axis=1).astype(np.int16)
    return (b1 @ (1 - b2).T + (1 - b1) @ b2.T).astype(np.int32)


def _rot_bin(rot):
    rot = np.float32(rot)
    if rot < 0.0:
        rot = np.float32(rot + np.float32(360.0))
    b = int(np.floor(float(np.float32(rot * np.float32(30 / 360.0))) + 0.5))   # roundf, exact in double
    return 0 if b == 30 else b


def _three_maxima(h):
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(h):
        if s > m1:
            m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
        elif s > m2:
            m3, m2, i3, i2 = m2, s, i2, i
        elif s > m3:
            m3, i3 = s, i
    if np.float32(m2) < np.float32(0.1) * np.float32(m1):
        i2 = i3 = -1
    elif np.float32(m3) < np.float32(0.1) * np.float32(m1):
        i3 = -1
    return i1, i2, i3


def _py_sbb(k1, ok1, fv1, k2, ok2, fv2, ratio, check_ori, frame_overload):
    """Both overloads literally (nodes in std::map order, the common ones only matter)."""
    D = _table(k1["desc"], k2["desc"])
    n1, n2 = len(k1["x"]), len(k2["x"])
    m12 = [-1] * n1
    taken2 = [False] * n2
    hist = [[] for _ in range(30)]
    nm = 0
    for node in sorted(set(fv1) & set(fv2)):
        for i1 in fv1[node]:
            if not ok1[i1]:
                continue
            b1, bi, b2 = 256, -1, 256
            for i2 in fv2[node]:
                if taken2[i2] or (ok2 is not None and not ok2[i2]):
                    continue
                d = int(D[i1, i2])
                if d < b1:
                    b2, b1, bi = b1, d, i2
                elif d < b2:
                    b2 = d
            if (b1 <= 50) if frame_overload else (b1 < 50):
                if np.float32(b1) < np.float32(ratio) * np.float32(b2):
                    m12[i1] = bi
                    taken2[bi] = True
                    if check_ori:
                        hist[_rot_bin(np.float32(k1["angle"][i1]) - np.float32(k2["angle"][bi]))].append(i1)
                    nm += 1
    if check_ori:
        keep = _three_maxima([len(h) for h in hist])
        for b in range(30):
            if b not in keep:
                for i1 in hist[b]:
                    m12[i1] = -1
                    nm -= 1
    return nm, np.array(m12, np.int32)


@pytest.mark.parametrize("levelsup,check_ori", [(2, True), (2, False), (4, True)])
def test_oracle_matches_restatement(levelsup, check_ori):
    k1, k2, fv1, fv2 = _problem(levelsup)
    a1, a2 = O.featvec_arrays(fv1), O.featvec_arrays(fv2)
    # keyframe-frame: frame side carries no map-point condition; result keyed by frame feature
    n, mf = O.search_by_bow_frame(k1, k1["has_mp"], a1, k2, a2, 0.7, check_ori)
    rn, r12 = _py_sbb(k1, k1["has_mp"], fv1, k2, None, fv2, 0.7, check_ori, True)
    ref_f = np.full(len(k2["x"]), -1, np.int32)
    ref_f[r12[r12 >= 0]] = np.flatnonzero(r12 >= 0)
    assert n == rn and np.array_equal(mf, ref_f)
    n, m12 = O.search_by_bow_kf(k1, k1["has_mp"], a1, k2, k2["has_mp"], a2, 0.75, check_ori)
    rn, r12 = _py_sbb(k1, k1["has_mp"], fv1, k2, k2["has_mp"], fv2, 0.75, check_ori, False)
    assert n == rn and np.array_equal(m12, r12)
    assert n > 50


def _frame(k):
    from orb_slam2_amd import Frame
    kp = np.zeros(len(k["x"]), dtype=[("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                                      ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
    kp["x"], kp["y"], kp["angle"], kp["octave"] = k["x"], k["y"], k["angle"], k["octave"]
    return Frame(kp, k["desc"], k["W"], k["H"])


@pytest.mark.gpu
@pytest.mark.parametrize("levelsup", [2, 3, 4])
def test_search_by_bow_gpu_bit_exact(amd, levelsup):
    k1, k2, fv1, fv2 = _problem(levelsup, seed=10 + levelsup)
    a1, a2 = O.featvec_arrays(fv1), O.featvec_arrays(fv2)
    f1, f2 = _frame(k1), _frame(k2)
    for ratio, ori in ((0.7, True), (0.6, False), (0.9, True)):
        m = amd.ORBmatcher(ratio, ori)
        n, mf = m.SearchByBoW(f1, k1["has_mp"], fv1, f2, a2)
        rn, rf = O.search_by_bow_frame(k1, k1["has_mp"], a1, k2, a2, ratio, ori)
        assert n == rn and np.array_equal(mf, rf), (ratio, ori)
        n, m12 = m.SearchByBoWKF(f1, k1["has_mp"], a1, f2, k2["has_mp"], fv2)
        rn, r12 = O.search_by_bow_kf(k1, k1["has_mp"], a1, k2, k2["has_mp"], a2, ratio, ori)
        assert n == rn and np.array_equal(m12, r12), (ratio, ori)
        m.close()


@pytest.mark.gpu
def test_search_by_bow_gpu_edges(amd):
    k1, k2, fv1, fv2 = _problem(2, seed=3)
    f1, f2 = _frame(k1), _frame(k2)
    m = amd.ORBmatcher(0.7, True)
    n, mf = m.SearchByBoW(f1, k1["has_mp"], {}, f2, fv2)            # empty feature vector
    assert n == 0 and np.all(mf == -1)
    n, mf = m.SearchByBoW(f1, np.zeros(len(k1["x"]), np.uint8), fv1, f2, fv2)   # no good map points
    assert n == 0 and np.all(mf == -1)
    same = dict(fv1)
    n, m12 = m.SearchByBoWKF(f1, np.ones(len(k1["x"]), np.uint8), same, f1, np.ones(len(k1["x"]), np.uint8), same)
    rn, r12 = O.search_by_bow_kf(k1, np.ones(len(k1["x"]), np.uint8), O.featvec_arrays(same), k1,
                                 np.ones(len(k1["x"]), np.uint8), O.featvec_arrays(same), 0.7, True)
    assert n == rn and np.array_equal(m12, r12) and n > 0             # a keyframe against itself
    m.close()
