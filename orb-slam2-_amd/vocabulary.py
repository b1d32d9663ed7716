"""Host mirror of DBoW2's TemplatedVocabulary<FORB::TDescriptor, FORB> as ORB-SLAM2 uses it
(ORBVocabulary, R/include/ORBVocabulary.h; D/ = Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h),
with the per-descriptor tree descent on the GPU (csrc/bow.hip, orb_vocabulary_transform).

The vocabulary is held flattened — node 0 the root, node descriptors [n, 32], children as CSR in
m_nodes[i].children order, word id and weight per node — and uploaded once.  The loaders follow
loadFromTextFile (D/TemplatedVocabulary.h:1362-1450) and loadFromBinaryFile (:1478-1522); node
ids are file order and every node is appended to its parent's children in that order.  One
deliberate difference: the text loader's `while(!f.eof())` reads the empty line after a final
newline as one more node (parent and descriptor uninitialised); that line is skipped here.
"""
import ctypes as C
import struct

import numpy as np

from . import _abi

# WeightingType / ScoringType / LNorm (D/BowVector.h:31-55)
TF_IDF, TF, IDF, BINARY = 0, 1, 2, 3
L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = 0, 1, 2, 3, 4, 5
L1, L2 = 0, 1


class VocabularyStruct(C.Structure):
    _fields_ = [("n_nodes", C.c_int), ("L", C.c_int), ("desc", C.c_void_p), ("child_start", C.c_void_p),
                ("child_idx", C.c_void_p), ("word_id", C.c_void_p), ("weight", C.c_void_p)]


def _must_normalize(scoring):
    """ScoringObject::mustNormalize (D/ScoringObject.h:75-93): every scoring but DOT_PRODUCT
    normalises, L2_NORM with L2, the rest with L1."""
    return scoring != DOT_PRODUCT, (L2 if scoring == L2_NORM else L1)


def _seq_sum(x):
    """Left-to-right double sum (the reference's `norm += ...` loops); np.cumsum accumulates
    sequentially."""
    return float(np.cumsum(x)[-1]) if len(x) else 0.0


class ORBVocabulary:
    """TemplatedVocabulary<FORB::TDescriptor, FORB> (D/TemplatedVocabulary.h:52-445)."""

    def __init__(self, k=10, L=5, weighting=TF_IDF, scoring=L1_NORM, device=0):
        self.m_k, self.m_L, self.m_weighting, self.m_scoring = k, L, weighting, scoring
        self.device = device
        self.desc = np.zeros((1, 32), np.uint8)
        self.parent = np.zeros(1, np.int32)
        self.child_start = np.zeros(2, np.int32)
        self.child_idx = np.zeros(0, np.int32)
        self.word_id = np.zeros(1, np.int32)
        self.weight = np.zeros(1, np.float64)
        self.n_words = 0
        self._h = None

    # -- construction ---------------------------------------------------------------------------
    @classmethod
    def from_nodes(cls, parent, is_leaf, desc, weight, k, L, weighting=TF_IDF, scoring=L1_NORM, device=0):
        """Nodes 1..n-1 in file order (entry 0 of each array is the root's and ignored): parent
        id, leaf flag, descriptor, weight.  Word ids are assigned to leaves in node order, as the
        loaders do."""
        v = cls(k, L, weighting, scoring, device)
        v._set_nodes(np.asarray(parent, np.int64), np.asarray(is_leaf, bool), np.asarray(desc, np.uint8),
                     np.asarray(weight, np.float64))
        return v

    def _set_nodes(self, parent, is_leaf, desc, weight):
        n = len(parent)
        if n < 1 or desc.shape != (n, 32) or len(is_leaf) != n or len(weight) != n:
            raise ValueError("vocabulary node arrays disagree in length")
        par = parent[1:]
        if len(par) and (par.min() < 0 or np.any(par >= np.arange(1, n))):
            raise ValueError("every node's parent must precede it")
        order = np.argsort(par, kind="stable") + 1          # children grouped by parent, file order
        counts = np.bincount(par, minlength=n) if len(par) else np.zeros(n, np.int64)
        self.child_start = np.zeros(n + 1, np.int32)
        self.child_start[1:] = np.cumsum(counts)
        self.child_idx = order.astype(np.int32)
        leaf = is_leaf.copy()
        leaf[0] = False
        self.word_id = np.zeros(n, np.int32)
        self.word_id[leaf] = np.arange(int(leaf.sum()), dtype=np.int32)
        self.n_words = int(leaf.sum())
        self.parent = parent.astype(np.int32)
        self.desc = np.ascontiguousarray(desc)
        self.weight = np.ascontiguousarray(weight, np.float64)
        self._release()

    def loadFromTextFile(self, filename):
        """D/TemplatedVocabulary.h:1362-1450: header "k L scoring weighting", then one line per
        node: parent, isLeaf, 32 descriptor bytes, weight."""
        with open(filename, "r") as f:
            head = f.readline().split()
            if len(head) < 4:
                return False
            k, L, n1, n2 = (int(x) for x in head[:4])
            if k < 0 or k > 20 or L < 1 or L > 10 or n1 < 0 or n1 > 5 or n2 < 0 or n2 > 3:
                return False
            rows = [ln.split() for ln in f if ln.strip()]
        n = len(rows) + 1
        parent = np.zeros(n, np.int64)
        leaf = np.zeros(n, bool)
        desc = np.zeros((n, 32), np.uint8)
        weight = np.zeros(n, np.float64)
        for i, r in enumerate(rows, 1):
            parent[i] = int(r[0])
            leaf[i] = int(r[1]) > 0
            desc[i] = [int(x) for x in r[2:34]]
            weight[i] = float(r[34])
        self.m_k, self.m_L, self.m_scoring, self.m_weighting = k, L, n1, n2
        self._set_nodes(parent, leaf, desc, weight)
        return True

    def saveToTextFile(self, filename):
        """D/TemplatedVocabulary.h:1453-1473 (weights printed with repr, so a reload is exact)."""
        leaf = self.child_start[1:] == self.child_start[:-1]
        with open(filename, "w") as f:
            f.write(f"{self.m_k} {self.m_L}  {self.m_scoring} {self.m_weighting}\n")
            for i in range(1, len(self.parent)):
                d = " ".join(str(int(x)) for x in self.desc[i])
                f.write(f"{self.parent[i]} {1 if leaf[i] else 0} {d}  {float(self.weight[i])!r}\n")

    def loadFromBinaryFile(self, filename):
        """D/TemplatedVocabulary.h:1478-1522: u32 nb_nodes, u32 size_node, int k, L, scoring,
        weighting, then per node (size_node bytes): int parent, 32 descriptor bytes, float
        weight, leaf byte at offset 40.  Exactly nb_nodes records are read: the reference's
        `while(!f.eof())` loop handles one more (stale buffer, m_nodes[nb_nodes + 1]) after the
        last, writing past the node array."""
        with open(filename, "rb") as f:
            blob = f.read()
        nb, size_node, k, L, sc, wt = struct.unpack_from("<IIiiii", blob, 0)
        body = np.frombuffer(blob, np.uint8, offset=24)
        cnt = min(nb, len(body) // size_node)
        recs = body[:cnt * size_node].reshape(cnt, size_node)
        n = cnt + 1
        parent = np.zeros(n, np.int64)
        parent[1:] = recs[:, 0:4].copy().view("<i4")[:, 0]
        desc = np.zeros((n, 32), np.uint8)
        desc[1:] = recs[:, 4:36]
        weight = np.zeros(n, np.float64)
        weight[1:] = recs[:, 36:40].copy().view("<f4")[:, 0]
        leaf = np.zeros(n, bool)
        leaf[1:] = recs[:, 40] != 0
        self.m_k, self.m_L, self.m_scoring, self.m_weighting = k, L, sc, wt
        self._set_nodes(parent, leaf, desc, weight)
        return True

    # -- queries ---------------------------------------------------------------------------------
    def size(self):
        return self.n_words

    def empty(self):
        return self.n_words == 0

    def getDepthLevels(self):
        return self.m_L

    def getBranchingFactor(self):
        return self.m_k

    # -- GPU handle ------------------------------------------------------------------------------
    def _handle(self):
        if self._h is None:
            lib = _abi.lib()
            _abi.sig(lib.orb_vocabulary_create, [C.c_int, C.c_void_p, C.c_void_p], C.c_int)
            s = VocabularyStruct(len(self.parent), self.m_L, _abi.ptr(self.desc), _abi.ptr(self.child_start),
                                 _abi.ptr(self.child_idx), _abi.ptr(self.word_id), _abi.ptr(self.weight))
            h = C.c_void_p()
            _abi.check("orb_vocabulary_create", lib.orb_vocabulary_create(self.device, C.byref(s), C.byref(h)))
            self._h = h
        return self._h

    def _release(self):
        if self._h is not None:
            lib = _abi.lib()
            _abi.sig(lib.orb_vocabulary_destroy, [C.c_void_p], None)
            lib.orb_vocabulary_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    # -- transform -------------------------------------------------------------------------------
    def transform_words(self, features, levelsup=0):
        """transform(feature, word_id, weight, &nid, levelsup) (D/TemplatedVocabulary.h:1242-1283)
        for every row of features ([n, 32] uint8) on the GPU: (word ids, weights, node ids)."""
        f = np.ascontiguousarray(np.asarray(features, np.uint8).reshape(-1, 32))
        n = len(f)
        wid = np.zeros(n, np.int32)
        w = np.zeros(n, np.float64)
        nid = np.zeros(n, np.int32)
        if n:
            lib = _abi.lib()
            _abi.sig(lib.orb_vocabulary_transform, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                                     C.c_void_p, C.c_void_p], C.c_int)
            _abi.check("orb_vocabulary_transform",
                       lib.orb_vocabulary_transform(self._handle(), _abi.ptr(f), n, levelsup, _abi.ptr(wid),
                                                    _abi.ptr(w), _abi.ptr(nid)))
        return wid, w, nid

    def transform(self, features, levelsup=0):
        """transform(features, BowVector& v, FeatureVector& fv, levelsup)
        (D/TemplatedVocabulary.h:1151-1218): returns (BowVector, FeatureVector) as dicts in
        std::map order — word id -> value, node id -> feature indices."""
        if self.empty():
            return {}, {}
        wid, w, nid = self.transform_words(features, levelsup)
        must, norm = _must_normalize(self.m_scoring)
        keep = np.flatnonzero(w > 0)                    # not stopped
        fv = {}
        for node in np.unique(nid[keep]):               # FeatureVector::addFeature, feature order
            fv[int(node)] = [int(i) for i in keep[nid[keep] == node]]
        order = keep[np.lexsort((keep, wid[keep]))]     # by word, feature order within a word
        words, first, counts = np.unique(wid[order], return_index=True, return_counts=True)
        vals = w[order[first]].copy()
        if self.m_weighting in (TF, TF_IDF):            # BowVector::addWeight, in feature order
            for g in np.flatnonzero(counts > 1):
                vals[g] = _seq_sum(w[order[first[g]:first[g] + counts[g]]])
            if len(vals) and not must:
                vals = vals / float(len(vals))
        # IDF / BINARY: addIfNotExist keeps the first feature's weight (vals already is that)
        if must and len(vals):
            s = _seq_sum(np.abs(vals)) if norm == L1 else float(np.sqrt(_seq_sum(vals * vals)))
            if s > 0.0:
                vals = vals / s
        return {int(a): float(b) for a, b in zip(words, vals)}, fv

    def score(self, v1, v2):
        """L1Scoring::score (D/ScoringObject.cpp:23-67) — the scoring ORBvoc uses: over the common
        words in ascending order, sum |vi - wi| - |vi| - |wi|, then -score / 2."""
        if self.m_scoring != L1_NORM:
            raise NotImplementedError("only the L1_NORM scoring ORBvoc.txt uses is mirrored")
        s = 0.0
        for wd in sorted(set(v1) & set(v2)):
            vi, wi = v1[wd], v2[wd]
            s += abs(vi - wi) - abs(vi) - abs(wi)
        return -s / 2.0
