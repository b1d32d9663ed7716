"""The benchmark's own path against the oracle.

bench.py times `Pipe.step` (orb_extract_batch_device + orb_search_for_initialization_batch_device,
4 sequences x 256 frames, each on its own HIP stream, issued back to back so the streams run
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
    W, H, NF, S = 640, 480, 1000, 4
    B = 512 if match_stream else 1024   # the bench's default step: 4 x 256 frames
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


def _check_frames(tag, frames, kps_t, desc_t, cnt_t, p, n_threads=16):
    """Every frame's keypoints (all 7 fields) and descriptors bit-exact vs the oracle's
    ORBextractor::operator(); returns the oracle outputs (want_pyramid for the stereo check)."""
    from orb_slam2_amd import _abi
    KP = _abi.KEYPOINT_DTYPE
    with cf.ThreadPoolExecutor(min(n_threads, os.cpu_count() or 1)) as ex:
        refs = list(ex.map(lambda im: O.extract(p, im, want_pyramid=True), frames))
    cnt, kps, desc = cnt_t.cpu().numpy(), kps_t.cpu().numpy(), desc_t.cpu().numpy()
    for i, ref in enumerate(refs):
        n = int(cnt[i])
        assert n == len(ref["kps"]), f"{tag} frame {i}: {n} vs {len(ref['kps'])} keypoints"
        assert kps[i, :n].copy().view(KP).reshape(-1).tobytes() == ref["kps"].tobytes(), f"{tag} frame {i}: keypoints"
        assert np.array_equal(desc[i, :n], ref["desc"]), f"{tag} frame {i}: descriptors"
    return refs


def test_bench_kitti_leg_matches_oracle(amd):
    """BASELINE config 3 as bench.py's extras time it (kitti_sfi_leg: KITTI 00 geometry 1241x376,
    2000 feat, B = 64 HBM-resident frames through orb_extract_batch_device, then
    orb_search_for_initialization_batch_device over the 63 in-batch pairs): every frame and every
    pair bit-exact vs the oracle (R/src/ORBextractor.cpp:1120-1188, R/src/ORBmatcher.cpp:499-617),
    and both handles' overflow bits read 0 (the leg raises otherwise)."""
    bench = _bench()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    m = amd.ORBmatcher(0.9, True, device=0)
    W, H, B = 1241, 376, 64
    _, b, frames = bench.kitti_sfi_leg(amd, dev, m, B, steps=2, warmup=1)
    assert b["status"] == {"extractor": 0, "matcher": 0}
    p = O.params(2000)
    refs = _check_frames("kitti", frames, b["kps"], b["desc"], b["cnt"], p)
    nm, m12 = b["nm"].cpu().numpy(), b["m12"].cpu().numpy()
    for q in range(B - 1):
        r1, r2 = refs[q], refs[q + 1]
        fa, fb = O.FrameView(r1["kps"], r1["desc"], W, H), O.FrameView(r2["kps"], r2["desc"], W, H)
        prev = np.stack([r1["kps"]["x"], r1["kps"]["y"]], 1).astype(np.float32).reshape(-1)
        n_ref, m_ref, _ = O.search_for_initialization(fa, fb, prev, nnratio=0.9, window=100)
        assert int(nm[q]) == n_ref, f"kitti pair {q}: nmatches"
        assert np.array_equal(m12[q, :len(r1["kps"])], m_ref), f"kitti pair {q}: matches12"
    assert float(nm.mean()) > 100


@pytest.mark.parametrize("pairs", [list(range(8)), [13, 14, 15]])
def test_bench_config5_batch_matches_oracle(amd, pairs):
    """BASELINE config 5 as bench.py times it (config5_shard: EuRoC geometry 752x480, 1200 feat,
    a full 8-pair stereo batch, and a 3-pair shard of the next batch as one rank of a sharded run
    holds it): both images of every pair extracted in one orb_extract_batch_device call, then
    orb_compute_stereo_matches_batch_device; every frame's keypoints / descriptors and every pair's
    mvuRight / mvDepth / nstereo bit-exact vs the oracle (R/src/Frame.cpp:551-770), batch status 0."""
    bench = _bench()
    from orb_slam2_amd import synth
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    W, H, NF = 752, 480, 1200
    cv = synth.canvas(0x5EED0005, W, H)
    step, o = bench.config5_shard(amd, dev, cv, pairs)
    step()
    step()
    torch.cuda.synchronize(dev)
    assert bench.batch_status(o["ex"], None, "config 5 test") == {"extractor": 0, "matcher": 0}
    p = O.params(NF)
    refs = _check_frames("config5", o["frames"], o["kps"], o["desc"], o["cnt"], p)
    ur, dep, ns = o["ur"].cpu().numpy(), o["dep"].cpu().numpy(), o["ns"].cpu().numpy()
    for j in range(len(pairs)):
        a, bb = refs[2 * j], refs[2 * j + 1]
        n_ref, ur_ref, dep_ref = O.compute_stereo_matches(p, a, bb, bench.EUROC_MBF)
        nl = len(a["kps"])
        assert int(ns[j]) == n_ref, f"pair {pairs[j]}: nstereo"
        assert np.array_equal(ur[j, :nl], ur_ref), f"pair {pairs[j]}: mvuRight"
        assert np.array_equal(dep[j, :nl], dep_ref), f"pair {pairs[j]}: mvDepth"
        assert n_ref > 300


def test_pcie_pipelined_leg_outputs_match_oracle(amd):
    """bench.py's pipelined PCIe-inclusive leg (copy stream + two compute streams, results packed by
    orb_pack_rows_device straight into host-mapped memory, three output sets in rotation): every
    consumed batch's packed keypoints (all 7 fields), descriptors and matches12 equal the oracle's
    ORBextractor::operator() and SearchForInitialization over the batch's in-batch pairs — the
    events between the streams leave no race."""
    bench = _bench()
    from orb_slam2_amd import _abi, synth
    W, H, NF, B = 640, 480, 1000, 8
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    cv = synth.canvas(0x5EED0002, W, H)
    p = O.params(NF)
    KP = _abi.KEYPOINT_DTYPE
    seen = []

    def check(s, frames, offs, kp, desc, m12):
        with cf.ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
            refs = list(ex.map(lambda im: O.extract(p, im), list(frames)))
        for b, ref in enumerate(refs):
            a, e = int(offs[0, b]), int(offs[0, b + 1])
            assert e - a == len(ref["kps"]), f"batch {s} frame {b}: {e - a} vs {len(ref['kps'])} keypoints"
            assert kp[a:e].copy().view(KP).reshape(-1).tobytes() == ref["kps"].tobytes(), f"batch {s} frame {b}"
            assert np.array_equal(desc[a:e], ref["desc"]), f"batch {s} frame {b}: descriptors"
            assert int(offs[1, b]) == a
        for q in range(B - 1):
            r1, r2 = refs[q], refs[q + 1]
            fa = O.FrameView(r1["kps"], r1["desc"], W, H)
            fb = O.FrameView(r2["kps"], r2["desc"], W, H)
            prev = np.stack([r1["kps"]["x"], r1["kps"]["y"]], 1).astype(np.float32).reshape(-1)
            _, m_ref, _ = O.search_for_initialization(fa, fb, prev, nnratio=0.9, window=100)
            a, e = int(offs[2, q]), int(offs[2, q + 1])
            assert np.array_equal(m12[a:e], m_ref), f"batch {s} pair {q}: matches12"
        seen.append(s)

    r = bench._pcie_pipelined_leg(amd, dev, cv, W, H, NF, B, steps=5, warmup=2, check=check)
    assert sorted(seen) == list(range(7)) and r["frames_per_s"] > 0
