"""MapPoint::ComputeDistinctiveDescriptors: the C oracle against a numpy restatement of the
reference loop (CPU), and the gfx950 batch kernel bit-exact against the oracle (GPU)."""
import numpy as np
import pytest

import oracle_ref as O


def _np_ref(desc):
    """R/src/MapPoint.cpp:343-378 in numpy: full distance table, per-row sort, element
    0.5*(N-1), least median with strict <."""
    N = len(desc)
    if N == 0:
        return -1
    bits = np.unpackbits(desc, axis=1).astype(np.int32)
    D = (bits[:, None, :] != bits[None, :, :]).sum(-1)
    best, bi = np.iinfo(np.int32).max, 0
    for i in range(N):
        med = np.sort(D[i])[int(0.5 * (N - 1))]
        if med < best:
            best, bi = med, i
    return bi


def _lists(seed, n_points=200, max_n=40):
    rng = np.random.default_rng(seed)
    out = []
    for m in range(n_points):
        n = int(rng.integers(0, max_n + 1))
        base = rng.integers(0, 256, 32, dtype=np.uint8)
        # observations of one point: the base descriptor with a few flipped bits each
        d = np.repeat(base[None], n, 0)
        flips = rng.random((n, 256)) < rng.uniform(0.02, 0.2)
        d = np.packbits(np.unpackbits(d, axis=1) ^ flips.astype(np.uint8), axis=1)
        out.append(d)
    out.append(np.repeat(out[5][:1], 6, 0) if len(out[5]) else np.zeros((6, 32), np.uint8))   # all equal
    out.append(np.zeros((1, 32), np.uint8))                                                   # single
    return out


def test_oracle_matches_numpy_restatement():
    for d in _lists(1, n_points=60):
        assert O.distinctive_descriptor(d) == _np_ref(d)


@pytest.mark.gpu
def test_distinctive_descriptors_gpu_bit_exact(amd):
    lists = _lists(2)
    lists.append(np.random.default_rng(3).integers(0, 256, (1500, 32), dtype=np.uint8))   # > LDS rows: HBM path
    best, out = amd.ComputeDistinctiveDescriptors(lists)
    for d, b, o in zip(lists, best, out):
        r = O.distinctive_descriptor(d)
        assert b == r
        if r >= 0:
            assert np.array_equal(o, d[r])
