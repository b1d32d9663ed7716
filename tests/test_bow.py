"""DBoW2 TemplatedVocabulary::transform (ORB-SLAM2's Frame/KeyFrame::ComputeBoW): the C oracle
against a literal Python restatement of the reference loops, the host loaders and
BowVector/FeatureVector assembly (CPU), and the gfx950 descent kernel bit-exact against the
oracle, at test size and at the 10^6-word ORBvoc shape (GPU).  Parity anchor: the reference
ships no vocabulary file or golden transform output (Vocabulary/ holds only
bin_vocabulary.cpp), so the oracle is pinned by this restatement of
D/DBoW2/TemplatedVocabulary.h:1151-1283, BowVector.cpp:34-84 and FeatureVector.cpp:31-45."""
import struct

import numpy as np
import pytest

import oracle_ref as O


def _hamming(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def _py_transform(parent, leaf, desc, weight, L, features, levelsup):
    """Literal restatement: m_nodes with children lists in loader order, the do/while descent of
    TemplatedVocabulary.h:1242-1283, then the TF_IDF branch of :1151-1190 with std::map
    semantics (dict + sorted keys) and BowVector::normalize(L1)."""
    n = len(parent)
    children = [[] for _ in range(n)]
    word = [0] * n
    nw = 0
    for i in range(1, n):
        children[int(parent[i])].append(i)
        if leaf[i]:
            word[i] = nw
            nw += 1
    v, fv = {}, {}
    for i_feature, f in enumerate(features):
        nid_level = L - levelsup
        nid = 0
        final_id = 0
        current_level = 0
        while True:
            current_level += 1
            nodes = children[final_id]
            final_id = nodes[0]
            best_d = _hamming(f, desc[final_id])
            for c in nodes[1:]:
                d = _hamming(f, desc[c])
                if d < best_d:
                    best_d = d
                    final_id = c
            if current_level == nid_level:
                nid = final_id
            if not children[final_id]:
                break
        w = float(weight[final_id])
        wid = word[final_id]
        if w > 0:
            v[wid] = v[wid] + w if wid in v else w
            fv.setdefault(nid, []).append(i_feature)
    norm = 0.0
    for k in sorted(v):
        norm += abs(v[k])
    if norm > 0.0:
        v = {k: v[k] / norm for k in sorted(v)}
    return {k: v[k] for k in sorted(v)}, {k: fv[k] for k in sorted(fv)}


def _voc(L=3, k=6, seed=7, **kw):
    from orb_slam2_amd import synth
    return synth.vocabulary(k=k, L=L, seed=seed, **kw)


def _features(voc, n, seed=11):
    from orb_slam2_amd import synth
    f = synth.bow_features(voc[2], voc[1], n, seed=seed)
    f[: min(3, n)] = voc[2][1: min(3, n) + 1]        # exact node descriptors
    return f


@pytest.mark.parametrize("levelsup", [0, 1, 2, 3, 5])
def test_oracle_matches_literal_restatement(levelsup):
    L = 3
    voc = _voc(L=L, dup_frac=0.15, early_leaf=0.2, stop_frac=0.2)
    feats = _features(voc, 120)
    ov = O.OracleVocabulary(*voc, L)
    bow, fv = O.bow_transform(ov, feats, levelsup)
    rb, rf = _py_transform(*voc, L, feats, levelsup)
    assert list(bow) == list(rb) and list(fv) == list(rf)
    assert all(bow[k] == rb[k] for k in rb)          # bit-exact doubles
    assert fv == rf


def test_host_flattening_and_loaders(tmp_path):
    from orb_slam2_amd.vocabulary import ORBVocabulary
    parent, leaf, desc, weight = _voc(L=3, early_leaf=0.2)
    v = ORBVocabulary.from_nodes(parent, leaf, desc, weight, k=6, L=3)
    start, idx, wid = O.flatten_vocabulary(parent, leaf, desc, weight)
    assert np.array_equal(v.child_start, start) and np.array_equal(v.child_idx, idx)
    assert np.array_equal(v.word_id, wid) and v.size() == int(leaf[1:].sum())
    # text round trip (saveToTextFile / loadFromTextFile, with the trailing newline)
    p = tmp_path / "voc.txt"
    v.saveToTextFile(str(p))
    w = ORBVocabulary()
    assert w.loadFromTextFile(str(p))
    assert (w.m_k, w.m_L, w.m_scoring, w.m_weighting) == (6, 3, 0, 0)
    for a in ("child_start", "child_idx", "word_id", "desc", "weight"):
        assert np.array_equal(getattr(v, a), getattr(w, a)), a
    # binary layout of loadFromBinaryFile: header, then (int parent, 32 B, float weight, leaf byte)
    size_node = 4 + 32 + 4 + 1
    blob = bytearray(struct.pack("<IIiiii", len(parent) - 1, size_node, 6, 3, 0, 0))
    for i in range(1, len(parent)):
        blob += struct.pack("<i", int(parent[i])) + desc[i].tobytes() + struct.pack("<f", weight[i]) + \
            bytes([1 if leaf[i] else 0])
    b = tmp_path / "voc.bin"
    b.write_bytes(bytes(blob))
    u = ORBVocabulary()
    assert u.loadFromBinaryFile(str(b))
    assert np.array_equal(u.child_idx, idx) and np.array_equal(u.word_id, wid)
    assert np.array_equal(u.weight, weight.astype(np.float32).astype(np.float64))
    # malformed header is refused like the reference loader
    bad = tmp_path / "bad.txt"
    bad.write_text("30 6 0 0\n")
    assert not ORBVocabulary().loadFromTextFile(str(bad))


def test_host_assembly_matches_oracle():
    """ORBVocabulary.transform's BowVector / FeatureVector assembly, fed the oracle's per-feature
    descent (no GPU here), against oracle_bow_transform."""
    from orb_slam2_amd.vocabulary import ORBVocabulary
    L = 4
    voc = _voc(L=L, k=5, dup_frac=0.1, stop_frac=0.15)
    feats = _features(voc, 600)
    ov = O.OracleVocabulary(*voc, L)
    v = ORBVocabulary.from_nodes(*voc, k=5, L=L)
    v.transform_words = lambda f, levelsup=0: O.vocab_transform(ov, f, levelsup)
    for levelsup in (0, 2, 4):
        bow, fv = v.transform(feats, levelsup)
        rb, rf = O.bow_transform(ov, feats, levelsup)
        assert list(bow) == list(rb) and all(bow[k] == rb[k] for k in rb) and fv == rf
    b1, _ = v.transform(feats[:300], 4)
    b2, _ = v.transform(feats[200:], 4)
    s = v.score(b1, b2)
    assert 0.0 < s < 1.0 and v.score(b1, b1) == pytest.approx(1.0)


@pytest.mark.gpu
def test_vocab_transform_gpu_bit_exact(amd):
    L = 4
    voc = _voc(L=L, k=8, dup_frac=0.08, early_leaf=0.1, stop_frac=0.1)
    feats = _features(voc, 5000)
    ov = O.OracleVocabulary(*voc, L)
    v = amd.ORBVocabulary.from_nodes(*voc, k=8, L=L)
    for levelsup in (0, 1, 2, 4, 6):
        wid, w, nid = v.transform_words(feats, levelsup)
        rw, rg, rn = O.vocab_transform(ov, feats, levelsup)
        assert np.array_equal(wid, rw) and np.array_equal(w, rg) and np.array_equal(nid, rn)
    bow, fv = v.transform(feats[:1000], 2)
    rb, rf = O.bow_transform(ov, feats[:1000], 2)
    assert list(bow) == list(rb) and all(bow[k] == rb[k] for k in rb) and fv == rf
    assert v.transform_words(np.zeros((0, 32), np.uint8), 4)[0].shape == (0,)


@pytest.mark.gpu
def test_vocab_transform_gpu_orbvoc_shape(amd):
    """k=10, L=6 (1,111,111 nodes, 10^6 words — the ORBvoc.txt shape), levelsup 4 as ComputeBoW."""
    L = 6
    voc = _voc(L=L, k=10, early_leaf=0.0, dup_frac=0.01)
    feats = _features(voc, 20000, seed=12)
    ov = O.OracleVocabulary(*voc, L)
    v = amd.ORBVocabulary.from_nodes(*voc, k=10, L=L)
    wid, w, nid = v.transform_words(feats, 4)
    rw, rg, rn = O.vocab_transform(ov, feats, 4)
    assert np.array_equal(wid, rw) and np.array_equal(w, rg) and np.array_equal(nid, rn)
