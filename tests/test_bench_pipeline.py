"""The benchmark's own path against the oracle.

bench.py times `Pipe.step` (orb_extract_batch_device + orb_search_for_initialization_batch_device,
4 sequences x 128 frames, each on its own HIP stream, issued back to back so the streams run
concurrently).  This test builds the same `Pipe` objects from bench.py on the same synthetic pool
(rank 0's seed), runs two steps exactly as the timed loop does, and checks after each step:

* every extracted frame's keypoints (all 7 cv::KeyPoint fields) and descriptors bit-exact against
  the oracle's ORBextractor::operator() (R/src/ORBextractor.cpp:1120-1188);
* every pair's matches12 and nmatches bit-exact against the oracle's
  ORBmatcher::SearchForInitialization(F_{t-1}, F_t, prev = F_{t-1}'s keypoints, window 100,
  nnratio 0.9, checkOri) (R/src/ORBmatcher.cpp:499-617), including the pair that spans two steps
  (row 0 = the previous step's last frame) and the first pair of step 0 (an empty F1);
* both handles' overflow bits (orb_extractor_batch_status, orb_matcher_batch_status) read 0.
"""
import concurrent.futures as cf
import os
import sys

import numpy as np
import pytest
import torch

import oracle_ref as O

pytestmark = pytest.mark.gpu


def _bench():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    import bench
    return bench


@pytest.mark.parametrize("match_stream", [False, True])
def test_bench_pipeline_matches_oracle(amd, match_stream):
    bench = _bench()
    from orb_slam2_amd import _abi, synth
    W, H, NF, B, S = 640, 480, 1000, 512, 4
    Bs = B // S
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    cv = synth.canvas(0x5EED0002, W, H)                      # bench.py main(), rank 0
    pool_np = np.stack([synth.frame(cv, W, H, t) for t in range(B)])
    pool = torch.from_numpy(pool_np).to(dev)
    cap, _, _ = bench.bench_capacity(amd, 0, W, H, NF)
    pipes = [bench.Pipe(k, amd, dev, 0, pool, W, H, NF, B, Bs, cap, match_stream) for k in range(S)]
    KP = _abi.KEYPOINT_DTYPE

    p = O.params(NF)
    cache = {}

    def oracle(i):
        if i not in cache:
            cache[i] = O.extract(p, pool_np[i])
        return cache[i]

    n_threads = min(16, os.cpu_count() or 1)
    prev_last = [None] * S            # pool index of each sequence's last frame of the previous step
    checked_frames = checked_pairs = 0
    for s in range(3 if match_stream else 2):
        for q in pipes:               # the bench's step(s): every sequence issued, no sync between
            q.step(s)
        torch.cuda.synchronize(dev)
        for k, q in enumerate(pipes):
            ext_st, m_st = q.status()
            assert ext_st == 0 and m_st == 0, f"step {s} seq {k}: overflow bits extractor {ext_st} matcher {m_st}"
            snap = q.snapshot()
            a, b = q.frame_range(s)
            idx = list(range(a, b))
            with cf.ThreadPoolExecutor(n_threads) as pool_ex:
                refs = list(pool_ex.map(oracle, idx))
            for r, (i, ref) in enumerate(zip(idx, refs), start=1):
                n = int(snap["counts"][r])
                got = snap["kps"][r, :n].copy().view(KP).reshape(-1)
                assert n == len(ref["kps"]), f"step {s} seq {k} frame {i}: {n} vs {len(ref['kps'])} keypoints"
                assert got.tobytes() == ref["kps"].tobytes(), f"step {s} seq {k} frame {i}: keypoints"
                assert np.array_equal(snap["desc"][r, :n], ref["desc"]), f"step {s} seq {k} frame {i}: descriptors"
                checked_frames += 1
            # pairs: (row b, row b+1), row 0 = previous step's last frame (empty at step 0)
            rows = [prev_last[k]] + idx
            for bq in range(Bs):
                i1, i2 = rows[bq], rows[bq + 1]
                n1 = 0 if i1 is None else len(oracle(i1)["kps"])
                if i1 is None:
                    assert int(snap["nm"][bq]) == 0
                    continue
                r1, r2 = oracle(i1), oracle(i2)
                fa = O.FrameView(r1["kps"], r1["desc"], W, H)
                fb = O.FrameView(r2["kps"], r2["desc"], W, H)
                prev = np.stack([r1["kps"]["x"], r1["kps"]["y"]], 1).astype(np.float32).reshape(-1)
                n_ref, m_ref, _ = O.search_for_initialization(fa, fb, prev, nnratio=0.9, window=100)
                assert int(snap["nm"][bq]) == n_ref, f"step {s} seq {k} pair {bq}: nmatches"
                assert np.array_equal(snap["m12"][bq, :n1], m_ref), f"step {s} seq {k} pair {bq}: matches12"
                checked_pairs += 1
            prev_last[k] = idx[-1]
    steps = 3 if match_stream else 2
    assert checked_frames == steps * B and checked_pairs == steps * B - S
