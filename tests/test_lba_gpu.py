"""GPU local BA vs the CPU oracle (g2o semantics): same LM decisions, chi2 to
1e-9 relative, poses / points to 1e-5 (north_star tolerance), same erase set."""
import ctypes as C

import numpy as np
import pytest

import oracle_ref as O

pytestmark = pytest.mark.gpu


def _problem(amd, **kw):
    from orb_slam2_amd import synth
    return synth.ba_problem(**kw)


def _compare(ref, got, tol=1e-5):
    assert got["iterations"] == ref["iterations"], (got["iterations"], ref["iterations"])
    assert got["trials"] == ref["trials"]
    assert np.allclose(got["trace"][:, 0], ref["trace"][:, 0], rtol=1e-9, atol=0)
    assert np.allclose(got["trace"][:, 1], ref["trace"][:, 1], rtol=1e-9, atol=0)
    assert np.allclose(got["trace"][:, 2], ref["trace"][:, 2], rtol=1e-9, atol=0)
    assert np.abs(got["pose_q"] - ref["pose_q"]).max() < tol
    assert np.abs(got["pose_t"] - ref["pose_t"]).max() < tol
    assert np.abs(got["point_xyz"] - ref["point_xyz"]).max() < tol
    assert np.array_equal(got["edge_erase"], ref["edge_erase"])
    assert np.allclose(got["edge_chi2"], ref["edge_chi2"], rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("kw", [
    dict(),                                                   # config 4: 20 KF x 3000 points, mono
    dict(stereo_frac=0.5, seed=7),                            # mixed mono / stereo edges
    dict(n_local=8, n_fixed=2, n_points=500, seed=3),
    dict(n_local=30, n_fixed=0, n_points=4000, seed=11, outlier_frac=0.15),
    dict(n_local=30, n_fixed=4, n_points=400, seed=13, k_range=(17, 30)),   # landmarks seen by 17-30 KFs
    dict(stereo_frac=1.0, seed=19, n_points=2000),            # every edge stereo (EdgeStereoSE3ProjectXYZ)
    dict(n_local=2, n_fixed=1, n_points=300, seed=20, k_range=(2, 3)),      # two local KFs (one free pose)
    dict(n_local=21, n_fixed=4, n_points=2500, seed=26),      # 20 free poses: n = 120, the LDS-image limit
    dict(n_local=12, n_fixed=2, n_points=1500, seed=27, outlier_frac=0.4),  # many erased edges
])
def test_local_ba_matches_oracle(amd, kw):
    pb = _problem(amd, **kw)
    ref = O.lba_solve(pb)
    got = amd.LocalBA().solve(pb)
    kc = min(3, len(pb["Tcw"]) - 1)
    q0, _ = O.quat_from_Tcw(pb["Tcw"][kc])
    assert np.array_equal(got["init_q"][kc], q0)     # Converter::toSE3Quat parity
    _compare(ref, got)


def test_local_ba_fixed_iterations(amd):
    pb = _problem(amd, n_points=1500, seed=5)
    ref = O.lba_solve(pb, O.lba_options(fixed_iterations=True))
    from orb_slam2_amd import optimizer
    got = amd.LocalBA().solve(pb, optimizer.options(fixed_iterations=True))
    _compare(ref, got)


def test_stop_flag_before_start(amd):
    pb = _problem(amd, n_points=300, seed=2)
    flag = (C.c_uint8 * 1)(1)
    got = amd.LocalBA().solve(pb, stop=flag)
    assert got["aborted"] and got["iterations"] == (0, 0)


def test_bad_points_skip_outlier_pass(amd):
    pb = _problem(amd, n_points=800, seed=9)
    pb["point_bad"][::7] = 1
    ref = O.lba_solve(pb)
    got = amd.LocalBA().solve(pb)
    _compare(ref, got)


@pytest.mark.parametrize("n,seed", [(6, 0), (114, 1), (120, 2), (128, 3), (130, 4), (180, 5), (301, 6), (600, 7),
                                    (1194, 8), (2100, 9)])
def test_dense_solve_vs_numpy(amd, n, seed):
    """Reduced camera system solve (blocked MFMA LDL^T: the LDS image up to 128, the
    multi-workgroup k_ldlt_mw_* beyond; past 2048 the backward substitution takes the per-super-block
    launches instead of k_ldlt_mw_back) against a float64 numpy solve of the same SPD system:
    relative residual at f64 rounding level."""
    rng = np.random.default_rng(seed)
    G = rng.standard_normal((n, n + 8))
    S = G @ G.T + n * np.eye(n)
    b = rng.standard_normal(n)
    x = amd.LocalBA().dense_solve(S, b)
    ref = np.linalg.solve(S, b)
    assert np.abs(x - ref).max() <= 1e-10 * np.abs(ref).max()
    assert np.abs(S @ x - b).max() <= 1e-11 * np.abs(b).max() * n


@pytest.mark.parametrize("n,seed,env", [
    (7, 30, None), (125, 31, None),                          # odd n: k_ldlt_solve<true> (S in LDS)
    (114, 32, "ORB_LBA_LDLT_OLD"), (64, 33, "ORB_LBA_LDLT_OLD"),
    (130, 34, "ORB_LBA_LDLT_SINGLE"), (181, 35, "ORB_LBA_LDLT_SINGLE"),   # k_ldlt_solve<false>
])
def test_dense_solve_alt_kernels_vs_numpy(amd, monkeypatch, n, seed, env):
    """The A/B forms of the reduced solve (k_ldlt_solve<true> for odd n or ORB_LBA_LDLT_OLD=1,
    k_ldlt_solve<false> under ORB_LBA_LDLT_SINGLE=1): these panels store +W, so their MFMA
    trailing tiles negate it on load (a sign slip there once went untested)."""
    if env:
        monkeypatch.setenv(env, "1")
    rng = np.random.default_rng(seed)
    G = rng.standard_normal((n, n + 8))
    S = G @ G.T + n * np.eye(n)
    b = rng.standard_normal(n)
    x = amd.LocalBA().dense_solve(S, b)
    ref = np.linalg.solve(S, b)
    assert np.abs(x - ref).max() <= 1e-10 * np.abs(ref).max()
    assert np.abs(S @ x - b).max() <= 1e-11 * np.abs(b).max() * n


@pytest.mark.parametrize("env", ["ORB_LBA_LDLT_OLD", "ORB_LBA_LDLT_SINGLE"])
def test_local_ba_alt_ldlt_matches_oracle(amd, monkeypatch, env):
    """Local BA through the A/B reduced-solve kernels: the same LM decisions as the oracle
    (config 4 under ORB_LBA_LDLT_OLD; 30 free poses, n = 180, under ORB_LBA_LDLT_SINGLE)."""
    monkeypatch.setenv(env, "1")
    kw = dict() if env == "ORB_LBA_LDLT_OLD" else dict(n_local=30, n_fixed=2, n_points=3000, seed=36)
    pb = _problem(amd, **kw)
    ref = O.lba_solve(pb)
    got = amd.LocalBA().solve(pb)
    _compare(ref, got)


def test_dense_solve_zero_pivot_fails(amd):
    S = np.eye(20)
    S[7, 7] = 0.0
    with pytest.raises(amd._abi.OrbError):
        amd.LocalBA().dense_solve(S, np.ones(20))


@pytest.mark.parametrize("stop_after", [0, 1, 3, 4, 7, 10, 13, 18])
def test_stop_after_trials_matches_oracle(amd, stop_after):
    """mbAbortBA raised at a reproducible point: terminate() true once the solve has run
    `stop_after` LM trials.  g2o samples it after every trial (levenberg.cpp:149), before every
    iteration (sparse_optimizer.cpp:376) and before the second optimize (Optimizer.cpp:792-796);
    the device's decision kernel samples at the same points, so decisions, estimates and the
    erase set equal the oracle stopped at the same trial."""
    pb = _problem(amd, n_local=12, n_fixed=2, n_points=1200, seed=31, outlier_frac=0.2)
    ref = O.lba_solve(pb, stop_after_trials=stop_after)
    ctx = amd.LocalBA()
    ctx.debug_stop_after_trials(stop_after)
    got = ctx.solve(pb)
    assert not got["aborted"]
    _compare(ref, got)            # iterations and trials equal the oracle's, stopped at the same trial
    assert got["trials"] == ref["trials"] and got["iterations"] == ref["iterations"]
    full = O.lba_solve(pb)
    if stop_after < full["trials"]:
        assert sum(got["iterations"]) < sum(full["iterations"]) or got["trials"] < full["trials"]


def test_stop_flag_raised_mid_solve_by_host_thread(amd):
    """The Tracking thread's InterruptBA (R/src/Tracking.cpp:1411) arrives while the solve runs:
    the LM loop stops at the next trial boundary, skips the second optimize() and still writes
    back; the result equals the oracle stopped after the same number of trials."""
    import threading
    import time
    pb = _problem(amd, n_local=30, n_fixed=4, n_points=12000, seed=33, outlier_frac=0.1)
    ctx = amd.LocalBA()
    ctx.solve(pb)                                    # warm-up (code objects, arena)
    t0 = time.perf_counter()
    full = ctx.solve(pb)
    t_full = time.perf_counter() - t0
    flag = (C.c_uint8 * 1)(0)
    timer = threading.Timer(t_full / 4, lambda: C.memset(flag, 1, 1))
    timer.start()
    got = ctx.solve(pb, stop=flag)
    timer.join()
    assert not got["aborted"]
    assert got["trials"] <= full["trials"]
    ref = O.lba_solve(pb, stop_after_trials=got["trials"])
    _compare(ref, got)


def test_lba_rejects_out_of_range_edges(amd):
    """lba_solve validates every edge index before touching host or device memory."""
    pb = _problem(amd, n_points=200, seed=4)
    bad = dict(pb)
    bad["edge_point"] = pb["edge_point"].copy()
    bad["edge_point"][5] = len(pb["point_xyz"])
    with pytest.raises(amd._abi.OrbError):
        amd.LocalBA().solve(bad)
    bad = dict(pb)
    bad["edge_pose"] = pb["edge_pose"].copy()
    bad["edge_pose"][0] = -1
    with pytest.raises(amd._abi.OrbError):
        amd.LocalBA().solve(bad)


def test_lba_coerces_field_dtypes(amd):
    """int64 edge indices and float32 observations are converted to the header's C types."""
    pb = _problem(amd, n_points=300, seed=6)
    ref = amd.LocalBA().solve(pb)
    alt = dict(pb)
    alt["edge_point"] = pb["edge_point"].astype(np.int64)
    alt["edge_pose"] = pb["edge_pose"].astype(np.int64)
    got = amd.LocalBA().solve(alt)
    assert got["iterations"] == ref["iterations"] and got["trials"] == ref["trials"]
    assert np.array_equal(got["point_xyz"], ref["point_xyz"]) and np.array_equal(got["pose_q"], ref["pose_q"])


def test_stop_after_rejected_trial(amd):
    """A stop inside a trial loop that is still open (its first trial was rejected, rho < 0).
    Near convergence the sign of rho is decided by the last bits of the chi2 sums, so such
    rejections do not line up with the oracle's; the semantics are therefore
    checked against the GPU's own bitwise-reproducible runs: stopped after the rejected trial,
    the solve counts that iteration, records lambda * ni and qmax 1 for it, keeps the popped
    estimates — bitwise those of the solve that ends just before the iteration — and the
    earlier trace rows equal the unstopped solve's."""
    from orb_slam2_amd import optimizer
    pb = _problem(amd, n_local=12, n_fixed=2, n_points=1200, seed=31, outlier_frac=0.2)
    full = amd.LocalBA().solve(pb, optimizer.options(5, 40, fixed_iterations=True))
    qmax = full["trace"][:, 3].astype(int)
    ks = [k for k in range(5, len(qmax)) if qmax[k] >= 2]
    assert ks, "this problem has rejected trials in the second round"
    k = ks[0]
    before = int(qmax[:k].sum())
    ctx = amd.LocalBA()
    ctx.debug_stop_after_trials(before + 1)
    got = ctx.solve(pb, optimizer.options(5, 40, fixed_iterations=True))
    assert got["iterations"] == (5, k - 5 + 1) and got["trials"] == before + 1
    assert np.array_equal(got["trace"][:k], full["trace"][:k])
    assert got["trace"][k, 0] == full["trace"][k, 0] and got["trace"][k, 1] == full["trace"][k, 0]
    assert got["trace"][k, 3] == 1 and got["trace"][k, 2] > full["trace"][k - 1, 2]
    upto = amd.LocalBA().solve(pb, optimizer.options(5, k - 5, fixed_iterations=True))
    assert np.array_equal(got["pose_q"], upto["pose_q"]) and np.array_equal(got["point_xyz"], upto["point_xyz"])


def test_local_ba_bitwise_reproducible(amd):
    """Every reduction of the LM pipeline has a fixed order and no two threads store the same
    element (k_schur_pairs keeps a diagonal block's upper triangle only): repeated solves on one
    context and on fresh contexts give bitwise identical estimates, traces and chi2."""
    pb = _problem(amd, n_points=600, seed=6, stereo_frac=0.3)
    ctx = amd.LocalBA()
    runs = [ctx.solve(pb) for _ in range(3)] + [amd.LocalBA().solve(pb) for _ in range(2)]
    for r in runs[1:]:
        for k in ("pose_q", "pose_t", "point_xyz", "edge_chi2", "trace", "edge_erase"):
            assert np.array_equal(r[k], runs[0][k]), k


def test_repeated_solves_bitwise_identical(amd):
    """Every reduction of the LM loop has a fixed order, so repeated solves (fresh and reused
    contexts, cached slot graphs) are bitwise identical — including fixed-iteration solves whose
    rejected trials end iterations, where a pop and the next linearisation share one launch."""
    from orb_slam2_amd import optimizer
    pb = _problem(amd, n_local=12, n_fixed=2, n_points=1200, seed=31, outlier_frac=0.2)
    opts = optimizer.options(5, 40, fixed_iterations=True)
    ref = amd.LocalBA().solve(pb, opts)
    assert (ref["trace"][:, 3] >= 2).any(), "the problem has rejected trials"
    ctx = amd.LocalBA()
    for r in [amd.LocalBA().solve(pb, opts)] + [ctx.solve(pb, opts) for _ in range(3)]:
        assert np.array_equal(r["trace"], ref["trace"])
        assert np.array_equal(r["pose_q"], ref["pose_q"]) and np.array_equal(r["point_xyz"], ref["point_xyz"])
        assert np.array_equal(r["edge_erase"], ref["edge_erase"])


@pytest.mark.parametrize("kw,shuffle_ids,global_ba", [
    (dict(), False, False),                                               # config 4
    (dict(stereo_frac=0.5, seed=7), True, False),                         # ids out of index order
    (dict(n_local=30, n_fixed=0, n_points=4000, seed=11), False, False),
    (dict(n_local=8, n_fixed=2, n_points=500, seed=3), True, True),       # Optimizer::BundleAdjustment
    # landmarks seen by 17-30 keyframes (k_struct_ptsort's insertion-sort path), edges shuffled
    (dict(n_local=30, n_fixed=4, n_points=400, seed=13, k_range=(17, 30), shuffle_edges=True), True, False),
])
def test_device_structure_matches_host_build(amd, monkeypatch, kw, shuffle_ids, global_ba):
    """The single-process solver builds the edge-level block structure on the device
    (k_struct_*): ORB_LBA_CHECK_STRUCT compares every array with the host build
    (csrc/lba_host.h) inside the call, and the solve equals the host-built one bitwise."""
    kw = dict(kw)
    shuffle_edges = kw.pop("shuffle_edges", False)
    pb = _problem(amd, **kw)
    if shuffle_edges:   # the edge order is the caller's: no grouping by landmark
        perm = np.random.default_rng(2).permutation(len(pb["edge_point"]))
        pb = {k: (v[perm] if k.startswith("edge_") else v) for k, v in pb.items()}
        assert np.bincount(pb["edge_point"]).max() > 16
    if shuffle_ids:   # g2o orders the Hessian blocks by vertex id, not by index
        rng = np.random.default_rng(1)
        pb = dict(pb)
        pb["pose_id"] = rng.permutation(len(pb["pose_id"])).astype(np.int64) * 3 + 1
        pb["point_id"] = rng.permutation(len(pb["point_id"])).astype(np.int64) + 1000
    monkeypatch.setenv("ORB_LBA_CHECK_STRUCT", "1")
    dev = amd.LocalBA().solve(pb, global_ba=global_ba)
    monkeypatch.delenv("ORB_LBA_CHECK_STRUCT")
    monkeypatch.setenv("ORB_LBA_HOST_STRUCT", "1")
    host = amd.LocalBA().solve(pb, global_ba=global_ba)
    for k in ("pose_q", "pose_t", "point_xyz", "edge_chi2", "trace", "edge_erase"):
        assert np.array_equal(dev[k], host[k]), k


@pytest.mark.parametrize("kw", [
    dict(n_local=60, n_fixed=4, n_points=8000, seed=21),                     # 6P = 354: multi-workgroup LDL^T
    dict(n_local=60, n_fixed=4, n_points=8000, seed=22, stereo_frac=0.5),
    dict(n_local=200, n_fixed=4, n_points=100000, seed=23),                  # SURVEY 8d's scaled config: 6P = 1194
])
def test_scaled_local_ba_matches_oracle(amd, kw):
    """Local BA windows beyond the LDS image (more than 21 free keyframes, R/src/Optimizer.cpp:569-625
    bounds the window only by covisibility): a corridor of keyframes with banded covisibility,
    the fused slots with the multi-workgroup reduced solve and the pair-list Schur complement,
    within the oracle's tolerances (identical LM decisions, chi2 trace 1e-9, estimates 1e-5)."""
    from orb_slam2_amd import synth
    pb = synth.ba_problem_corridor(**kw)
    ref = O.lba_solve(pb)
    got = amd.LocalBA().solve(pb)
    _compare(ref, got)


def test_scaled_local_ba_bitwise_reproducible(amd):
    """The multi-workgroup solve and the pair-list Schur keep every reduction order fixed."""
    from orb_slam2_amd import synth
    pb = synth.ba_problem_corridor(n_local=40, n_fixed=2, n_points=4000, seed=24, stereo_frac=0.3)
    ctx = amd.LocalBA()
    runs = [ctx.solve(pb) for _ in range(2)] + [amd.LocalBA().solve(pb)]
    for r in runs[1:]:
        for k in ("pose_q", "pose_t", "point_xyz", "edge_chi2", "trace", "edge_erase"):
            assert np.array_equal(r[k], runs[0][k]), k


@pytest.mark.parametrize("shuffle", [False, True])
def test_mw_envelope_bitwise_matches_dense(amd, monkeypatch, shuffle):
    """The multi-workgroup LDL^T skips the trailing tiles, panel row groups and back-substitution
    row blocks left of the reduced matrix's envelope (k_mw_envelope), and runs each panel's
    trailing update with the next panel's factorisation in one launch (k_ldlt_mw_step).  The
    skipped work adds exact zeros and the fused panel forms the same MFMA tiles, so the solve is
    bitwise the dense two-launch passes' (ORB_LBA_MW_DENSE=1 ORB_LBA_MW_SPLIT=1) and the envelope's
    alone (ORB_LBA_MW_SPLIT=1) — on the corridor's band and on the same window with its keyframes
    in shuffled order (an irregular envelope), which also stays within the oracle's tolerances."""
    from orb_slam2_amd import synth
    pb = synth.ba_problem_corridor(n_local=40, n_fixed=2, n_points=4000, seed=26, stereo_frac=0.2)
    if shuffle:
        rng = np.random.default_rng(3)
        nk = len(pb["Tcw"])
        perm = rng.permutation(nk)
        inv = np.empty(nk, np.int64)
        inv[perm] = np.arange(nk)
        pb = dict(pb, Tcw=pb["Tcw"][perm], pose_fixed=pb["pose_fixed"][perm],
                  pose_id=np.arange(nk, dtype=np.int64), edge_pose=inv[pb["edge_pose"]].astype(np.int32))
    monkeypatch.setenv("ORB_LBA_MW_DENSE", "1")
    monkeypatch.setenv("ORB_LBA_MW_SPLIT", "1")
    dense = amd.LocalBA().solve(pb)
    monkeypatch.delenv("ORB_LBA_MW_DENSE")
    envelope = amd.LocalBA().solve(pb)
    monkeypatch.delenv("ORB_LBA_MW_SPLIT")
    fused = amd.LocalBA().solve(pb)
    for got in (envelope, fused):
        assert got["iterations"] == dense["iterations"] and got["trials"] == dense["trials"]
        for k in ("pose_q", "pose_t", "point_xyz", "edge_chi2", "trace", "edge_erase"):
            assert np.array_equal(got[k], dense[k]), k
    if shuffle:
        _compare(O.lba_solve(pb), fused)


@pytest.mark.parametrize("small", ["-1", "0", "64", "100000"])
def test_schur_pair_units_match_oracle(amd, monkeypatch, small):
    """k_schur_pairs' work units (k_pair_list): every off-diagonal pose pair sharing at most
    ORB_LBA_SMALL_PAIR landmarks takes one wave, the others (and the diagonal blocks) a workgroup.
    All workgroups (-1), all waves (100000) and mixed splits stay within the oracle's tolerances,
    with identical LM decisions, and each split is bitwise reproducible."""
    from orb_slam2_amd import synth
    monkeypatch.setenv("ORB_LBA_SMALL_PAIR", small)
    pb = synth.ba_problem_corridor(n_local=40, n_fixed=2, n_points=4000, seed=25, stereo_frac=0.2)
    got = amd.LocalBA().solve(pb)
    _compare(O.lba_solve(pb), got)
    again = amd.LocalBA().solve(pb)
    for k in ("pose_q", "pose_t", "point_xyz", "trace", "edge_erase"):
        assert np.array_equal(again[k], got[k]), k


@pytest.mark.parametrize("kw", [dict(), dict(stereo_frac=0.5, seed=7)])
def test_schur_mfma_mode_matches_oracle(amd, monkeypatch, kw):
    """ORB_LBA_SCHUR_MFMA=1: the Schur complement as the densified f64 MFMA GEMM S -= Y Y^T
    (k_schur_ymat / k_schur_gemm / k_schur_msum, the A/B of SURVEY 8d) within the oracle's
    tolerances, and bitwise reproducible."""
    monkeypatch.setenv("ORB_LBA_SCHUR_MFMA", "1")
    pb = _problem(amd, **kw)
    got = amd.LocalBA().solve(pb)
    _compare(O.lba_solve(pb), got)
    again = amd.LocalBA().solve(pb)
    assert np.array_equal(again["trace"], got["trace"]) and np.array_equal(again["point_xyz"], got["point_xyz"])
