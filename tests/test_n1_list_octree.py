"""N1 (DistributeOctTree tie-break, R/src/ORBextractor.cpp:736, 783-784): the std::list-of-heap-
nodes restatement (oracle/n1_list_octree.cpp) run with creation-order ties reproduces the oracle's
octree (oracle_distribute_octree) on every level of a frame, so the measured disagreement of
heap-address ties (tools/n1_disagreement.py, profiles/r02_n1_disagreement.json) is the tie-break
alone.  Heap-address mode is only checked for well-formedness: its result depends on allocator
state and pins nothing."""
import ctypes as C
import pathlib

import numpy as np
import pytest

import oracle_ref as O

ROOT = pathlib.Path(__file__).resolve().parents[1]
LIB = ROOT / "oracle" / "build" / "libn1_list_octree.so"


@pytest.mark.parametrize("W,H,NF,seed", [(640, 480, 1000, 0x5EED0002), (752, 480, 1200, 0x5EED0005)])
def test_list_octree_creation_order_matches_oracle(W, H, NF, seed):
    if not LIB.exists():
        pytest.skip("oracle/build/libn1_list_octree.so not built")
    from orb_slam2_amd import synth
    n1 = C.CDLL(str(LIB))
    n1.n1_list_octree.restype = C.c_int
    P = O.P
    p = O.params(NF)
    fpl = O.tables(p)["features_per_level"]
    ex = O.extract(p, synth.frame(synth.canvas(seed, W, H), W, H, 0), want_pyramid=True)
    lw, lh = ex["sizes"]
    offs = np.concatenate([[0], np.cumsum(lw.astype(np.int64) * lh)])
    for l in range(len(lw)):
        img = np.ascontiguousarray(ex["pyramid"][offs[l]:offs[l + 1]].reshape(lh[l], lw[l]))
        cap = int(lw[l]) * int(lh[l]) // 4 + 64
        kx, ky, kr = (np.zeros(cap, np.float32) for _ in range(3))
        n = O.lib().oracle_level_keys(C.byref(p), P(img), int(lw[l]), int(lh[l]), P(kx), P(ky), P(kr), cap)
        kx, ky, kr = kx[:n], ky[:n], kr[:n]
        maxX, maxY = int(lw[l]) - 19 + 3, int(lh[l]) - 19 + 3
        want = O.distribute_octree(kx, ky, kr, 16, maxX, 16, maxY, int(fpl[l]))
        got = np.zeros(n + 1, np.int32)
        ng = n1.n1_list_octree(P(kx), P(ky), P(kr), n, 16, maxX, 16, maxY, int(fpl[l]), 1, P(got))
        assert np.array_equal(got[:ng], want), f"level {l}"
        heap = np.zeros(n + 1, np.int32)
        nh = n1.n1_list_octree(P(kx), P(ky), P(kr), n, 16, maxX, 16, maxY, int(fpl[l]), 0, P(heap))
        # (the tie-break can change which nodes are split, so the count may differ by a few)
        assert 0 < nh <= n and len(set(heap[:nh].tolist())) == nh and heap[:nh].max() < n
