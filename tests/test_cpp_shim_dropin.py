"""The per-frame and LocalMapping rows of SURVEY §8f through the compiled C++ drop-in path
(tests/cpp/shim_caller.cpp over include/orbslam2_amd_shim.hpp, mock reference types), and the
§8b threading contract:

* Optimizer::PoseOptimization (R/src/Optimizer.cpp:306-535): edges gathered from the mock Frame's
  mvpMapPoints in keypoint order, mvbOutlier / SetPose / return value written back — identical to
  the Python binding of pose_optimize_batch, within the oracle's tolerances (1e-5) and with its
  outlier flags and count;
* Frame::ComputeStereoMatches (R/src/Frame.cpp:551-770) after two concurrent extractions (the
  stereo Frame constructor, :86-89): keypoints, descriptors, mvuRight, mvDepth bit-exact vs the
  oracle;
* ORBmatcher::Fuse (R/src/ORBmatcher.cpp:995-1154): the GPU matching step plus the shim's
  replace / add loop on mock map points, against a Python restatement of that loop driven by the
  oracle's matches;
* ORBmatcher::SearchForTriangulation (:785-983), the epipole derived by the shim from the mock
  keyframes' poses; SearchByBoW (keyframe-frame :220-372, keyframe-keyframe :632-760): bit-exact;
* the threading contract (SURVEY §8b, R/src/Frame.cpp:86-89, R/src/LocalMapping.cpp:94-95): two
  extractor handles on two threads, SearchForInitialization, PoseOptimization and
  LocalBundleAdjustment on three more, all at once and repeated — every repetition identical and
  every result equal to its single-threaded oracle check."""
import numpy as np
import pytest

import oracle_ref as O
from orb_slam2_amd import synth
from test_cpp_shim import GRID, _frame_arrays, _read, _run, _write, shim  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu
F32 = np.float32
# Camera.bf of R/Examples/Stereo/EuRoC.yaml / KITTI00-02.yaml as the float Frame::mbf
EUROC_BF, KITTI_BF = (float(F32(synth.CAMERAS[k]["bf"])) for k in ("EUROC", "KITTI00"))


# ------------------------------------------------------------------ PoseOptimization
INV_SIGMA2 = (F32(1.0) / np.array([F32(1.2) ** (2 * lv) for lv in range(8)], F32))


def _pose_inputs(frame, seed):
    """A mock Frame around one synth.pose_problems frame: the frame's edges at random keypoint
    positions among keypoints without a map point."""
    rng = np.random.default_rng(seed)
    E = len(frame["info"])
    n = E + E // 3
    pos = np.sort(rng.choice(n, E, replace=False))
    x, y = rng.uniform(0, 640, n).astype(F32), rng.uniform(0, 480, n).astype(F32)
    oc = rng.integers(0, 8, n).astype(np.int32)
    ur = np.full(n, -1, F32)
    has = np.zeros(n, np.uint8)
    xyz = np.zeros((n, 3), F32)
    x[pos], y[pos] = frame["obs"][:, 0].astype(F32), frame["obs"][:, 1].astype(F32)
    ur[pos] = frame["obs"][:, 2].astype(F32)
    oc[pos] = [int(np.argmin(np.abs(INV_SIGMA2.astype(np.float64) - i))) for i in frame["info"]]
    has[pos] = 1
    xyz[pos] = frame["xw"].astype(F32)
    arrays = (np.asarray(frame["Tcw"], F32).reshape(-1), x, y, oc, ur, has, xyz.reshape(-1), INV_SIGMA2,
              np.asarray(frame["cam"], F32))
    return arrays, pos


@pytest.mark.parametrize("kw", [dict(stereo_frac=0.4, seed=9), dict(n_points=60, outlier_frac=0.3, seed=2)])
def test_shim_pose_optimization(shim, tmp_path, amd, kw):
    from orb_slam2_amd import synth, optimizer as opt
    frames = synth.pose_problems(n_frames=2, **kw)
    for f, frame in enumerate(frames):
        # the shim reads the intrinsics from the Frame's float members (e->fx = pFrame->fx, R :366-369)
        frame = dict(frame, cam=tuple(float(np.float32(v)) for v in frame["cam"]))
        arrays, pos = _pose_inputs(frame, 100 + f)
        r, outp = _run(shim, "pose", tmp_path, *arrays)
        assert r.returncode == 0, r.stderr
        n, outl, T = _read(outp, np.int32, np.uint8, F32)
        got = amd.PoseOptimization([frame])[0]          # the Python binding: same library call
        ref = O.pose_optimization(frame)
        assert int(n[0]) == got["n_inliers"] == ref["n_inliers"]
        assert np.array_equal(outl[pos], got["outlier"]) and np.array_equal(outl[pos], ref["outlier"])
        rest = np.setdiff1d(np.arange(len(outl)), pos)
        assert np.all(outl[rest] == 1)                  # keypoints without a map point: untouched
        assert np.array_equal(T.reshape(4, 4), opt.pose_to_Tcw(got["pose_q"], got["pose_t"]))
        assert np.abs(T.reshape(4, 4) - opt.pose_to_Tcw(ref["pose_q"], ref["pose_t"])).max() < 1e-5


def test_shim_pose_optimization_too_few_edges(shim, tmp_path):
    """Below 3 correspondences (R :431-432): return 0, the pose untouched, the edges' flags reset."""
    from orb_slam2_amd import synth
    frame = synth.pose_problems(n_frames=1, n_points=2, seed=3)[0]
    arrays, pos = _pose_inputs(frame, 7)
    r, outp = _run(shim, "pose", tmp_path, *arrays)
    assert r.returncode == 0, r.stderr
    n, outl, T = _read(outp, np.int32, np.uint8, F32)
    assert int(n[0]) == 0 and np.all(outl[pos] == 0)
    assert np.array_equal(T, arrays[0])


# ------------------------------------------------------------------ stereo Frame
def _stereo_inputs(W, H, NF, seed, t, mbf):
    from orb_slam2_amd import synth
    cv = synth.canvas(seed, W, H)
    left, right = synth.stereo_pair(cv, W, H, t)
    return (np.array([W, H, NF], np.int32), left, right, np.array([mbf, 0.0], F32)), (left, right)


def _check_stereo(outp, imgs, NF, mbf):
    kl, dl, kr, dr, ur, dep = _read(outp, np.uint8, np.uint8, np.uint8, np.uint8, F32, F32)
    p = O.params(NF)
    a = O.extract(p, imgs[0], want_pyramid=True)
    b = O.extract(p, imgs[1], want_pyramid=True)
    assert np.array_equal(kl.view(O.KP_DTYPE), a["kps"]) and np.array_equal(dl.reshape(-1, 32), a["desc"])
    assert np.array_equal(kr.view(O.KP_DTYPE), b["kps"]) and np.array_equal(dr.reshape(-1, 32), b["desc"])
    n_ref, ur_ref, dep_ref = O.compute_stereo_matches(p, a, b, mbf)
    assert np.array_equal(ur, ur_ref) and np.array_equal(dep, dep_ref)
    assert int((ur >= 0).sum()) == n_ref and n_ref > 300


@pytest.mark.parametrize("W,H,NF,seed,mbf", [(752, 480, 1200, 0x5EED0005, EUROC_BF), (1241, 376, 2000, 0x5EED0003, KITTI_BF)])
def test_shim_stereo_frame(shim, tmp_path, W, H, NF, seed, mbf):
    arrays, imgs = _stereo_inputs(W, H, NF, seed, 2, mbf)
    r, outp = _run(shim, "stereo", tmp_path, *arrays)
    assert r.returncode == 0, r.stderr
    _check_stereo(outp, imgs, NF, mbf)


# ------------------------------------------------------------------ keyframes
def _kf_arrays(k, Tcw, Ow, cam, sf, isg, sg2, fv):
    """load_kf's input for a synth keyframe dict (x, y, angle, octave, desc, uright, W, H)."""
    n = len(k["x"])
    W, H = k["W"], k["H"]
    grid = np.array([0, 0, W, H, F32(64) / F32(W), F32(48) / F32(H)], F32)
    ur = k.get("uright")
    ur = np.full(n, -1, F32) if ur is None else np.asarray(ur, F32)
    T = np.eye(4, dtype=F32)
    T[:3, :4] = np.asarray(Tcw, F32)[:3, :4]
    nodes, start, idx = fv
    return (np.asarray(k["x"], F32), np.asarray(k["y"], F32), np.asarray(k["angle"], F32),
            np.asarray(k["octave"], np.int32), np.ascontiguousarray(k["desc"], np.uint8), ur, grid, T.reshape(-1),
            np.asarray(Ow, F32), np.asarray(cam, F32), np.array([np.log(F32(1.2))], F32), np.asarray(sf, F32),
            np.asarray(isg, F32), np.asarray(sg2, F32), np.asarray(nodes, np.uint32), np.asarray(start, np.int32),
            np.asarray(idx, np.int32))


SF = np.array([F32(1.2) ** lv for lv in range(8)], F32)
SG2 = (SF * SF).astype(F32)
ISG2 = (F32(1.0) / SG2).astype(F32)
EMPTY_FV = (np.zeros(0, np.uint32), np.zeros(1, np.int32), np.zeros(0, np.int32))


def _py_fuse_resolve(best, vec, n_slots, slot0, bad0, extra0):
    """The replace / add loop of R/src/ORBmatcher.cpp:1006-1150 on a one-keyframe map, in vector
    order, given the matching step's best keypoint per point (MapPoint::Replace as
    R/src/MapPoint.cpp:177-219 moves observations; only this keyframe is modelled)."""
    np_ = len(bad0)
    slots = [-1] * n_slots
    in_kf = [int(s) for s in slot0]
    for i, s in enumerate(slot0):
        if s >= 0:
            slots[s] = i
    bad, extra, repl = [bool(b) for b in bad0], [int(e) for e in extra0], [-1] * np_

    def obs(i):
        return extra[i] + (1 if in_kf[i] >= 0 else 0)

    def replace(a, b):          # a->Replace(b)
        if a == b:
            return
        bad[a], repl[a] = True, b
        if in_kf[a] >= 0:
            s = in_kf[a]
            in_kf[a] = -1
            if in_kf[b] < 0:
                slots[s] = b
                in_kf[b] = s
            else:
                slots[s] = -1
        extra[b] += extra[a]   # (the replaced point keeps its stale count, as the mock does)

    n_fused = 0
    for v in vec:
        if v < 0 or bad[v] or in_kf[v] >= 0 or best[v] < 0:
            continue
        b = int(best[v])
        q = slots[b]
        if q >= 0:
            if not bad[q]:
                if obs(q) > obs(v):
                    replace(v, q)
                else:
                    replace(q, v)
        else:
            in_kf[v] = b
            slots[b] = v
        n_fused += 1
    return n_fused, slots, bad, repl, in_kf, [obs(i) for i in range(np_)]


@pytest.mark.parametrize("seed,th", [(3, 3.0), (11, 5.0)])
def test_shim_fuse(shim, tmp_path, seed, th):
    from orb_slam2_amd import synth
    p = synth.fuse_problem(seed=seed)
    kf, kp = p["kf"], p["kp"]
    rng = np.random.default_rng(seed)
    nk, nm = len(kf["x"]), len(p["mp_valid"])
    # the keyframe's own points: 30 % of its keypoints (observation counts 0..5 elsewhere)
    own = np.flatnonzero(rng.random(nk) < 0.3)
    n_own = len(own)
    # vector entries: the synthetic points; an invalid one becomes NULL, a bad point or a point
    # already in the keyframe (a free slot), a few valid ones repeated later in the vector
    kind = np.where(p["mp_valid"] == 0, rng.integers(0, 3, nm), -1)
    free = np.setdiff1d(np.arange(nk), own)
    in_slot = np.full(nm, -1, np.int32)
    pick = rng.choice(free, int((kind == 2).sum()), replace=False)
    in_slot[kind == 2] = pick
    vec = [(-1 if kind[i] == 0 else i) for i in range(nm)]
    dup = rng.choice(np.flatnonzero(kind < 0), 25, replace=False)
    vec += [int(i) for i in dup]
    rng.shuffle(vec)
    np_ = nm + n_own
    xyz = np.zeros((np_, 3), F32); nrm = np.zeros((np_, 3), F32)
    mind = np.zeros(np_, F32); maxd = np.zeros(np_, F32); desc = np.zeros((np_, 32), np.uint8)
    xyz[:nm], nrm[:nm], mind[:nm], maxd[:nm], desc[:nm] = (p["mp_xyz"], p["mp_normal"], p["mp_min_dist"],
                                                          p["mp_max_dist"], p["mp_desc"])
    bad = np.zeros(np_, np.uint8)
    bad[:nm] = kind == 1
    bad[nm:] = rng.random(n_own) < 0.1          # some of the keyframe's points are bad
    extra = rng.integers(0, 6, np_).astype(np.int32)
    slot = np.concatenate([in_slot, own.astype(np.int32)])
    T = np.eye(4, dtype=F32)
    T[:3] = kp["Tcw"]
    kfa = _kf_arrays(kf, T, kp["Ow"], kp["cam"], kp["scale_factors"], kp["inv_level_sigma2"], SG2, EMPTY_FV)
    r, outp = _run(shim, "fuse", tmp_path, *kfa, xyz.reshape(-1), nrm.reshape(-1), mind, maxd, desc.reshape(-1), bad,
                   extra, slot, np.array(vec, np.int32), np.array([th], F32))
    assert r.returncode == 0, r.stderr
    n, slots, st = _read(outp, np.int32, np.int32, np.int32)
    # the matching step: the oracle on the points valid at the call (not NULL, not bad, not in pKF)
    q = dict(p)
    q["mp_valid"] = ((kind < 0) & (p["mp_valid"] != 0)).astype(np.uint8)
    best, _ = O.fuse(q, th)
    best_all = np.full(np_, -1, np.int32)
    best_all[:nm] = best
    rn, rslots, rbad, rrepl, rin, robs = _py_fuse_resolve(best_all, vec, nk, slot, bad, extra)
    st = st.reshape(-1, 4)
    assert int(n[0]) == rn and rn > 100
    assert np.array_equal(slots, rslots)
    assert np.array_equal(st[:, 0], np.array(rbad, np.int32)) and np.array_equal(st[:, 1], rrepl)
    assert np.array_equal(st[:, 2], rin) and np.array_equal(st[:, 3], robs)
    assert (st[:, 1] >= 0).sum() > 10             # both replace directions exercised
    assert any(rslots[s] < nm and rslots[s] >= 0 and slot[rslots[s]] < 0 for s in range(nk))   # adds


def _epipole(R1, t1, R2, t2, cam):
    """ex, ey of R/src/ORBmatcher.cpp:791-797 as the shim evaluates them: C = -R1^T t1 (the mock
    keyframe's GetCameraCenter), C2 = R2*C + t2 with the double-accumulated OpenCV float GEMM."""
    C = (-(R1.astype(np.float64).T @ t1.astype(np.float64))).astype(F32)
    C2 = (R2.astype(np.float64) @ C.astype(np.float64) + t2.astype(np.float64)).astype(F32)
    invz = F32(1.0) / C2[2]
    fx, fy, cx, cy = (F32(v) for v in cam[:4])
    return F32(F32(fx * C2[0]) * invz) + cx, F32(F32(fy * C2[1]) * invz) + cy, C


@pytest.mark.parametrize("only_stereo,check_ori", [(False, True), (True, False)])
def test_shim_search_for_triangulation(shim, tmp_path, only_stereo, check_ori):
    from orb_slam2_amd import synth
    p = synth.triangulation_problem()
    cam = np.array(list(synth.TUM1) + [synth.KITTI_BF], F32)
    ex, ey, C1 = _epipole(p["R1"], p["t1"], p["R2"], p["t2"], cam)
    q = dict(p, ex=float(ex), ey=float(ey))
    n_ref, m_ref = O.search_for_triangulation(q, only_stereo, check_ori)
    ins = []
    for k, R, t, C in ((p["kf1"], p["R1"], p["t1"], C1), (p["kf2"], p["R2"], p["t2"], None)):
        T = np.eye(4, dtype=F32)
        T[:3, :3], T[:3, 3] = R, t
        Ow = C if C is not None else (-(R.astype(np.float64).T @ t.astype(np.float64))).astype(F32)
        ins += list(_kf_arrays(k, T, Ow, cam, p["scale_factors"], ISG2, p["level_sigma2"],
                               (k["nodes"], k["start"], k["fidx"])))
        ins.append(np.where(k["has_mp"] != 0, 0, -1).astype(np.int32))
    r, outp = _run(shim, "sft", tmp_path, *ins, p["F12"].reshape(-1).astype(F32),
                   np.array([int(only_stereo), int(check_ori)], np.int32))
    assert r.returncode == 0, r.stderr
    n, pairs = _read(outp, np.int32, np.int32)
    want = np.stack([np.flatnonzero(m_ref >= 0), m_ref[m_ref >= 0]], 1).astype(np.int32)
    assert int(n[0]) == n_ref and np.array_equal(pairs.reshape(-1, 2), want)
    assert n_ref > (10 if only_stereo else 50)


def _bow(levelsup=3, seed=12):
    from test_search_by_bow import _problem
    return _problem(levelsup, seed=seed)


def _slot_kinds(has_mp, rng):
    """-1 no map point, 0 a good one, 1 a bad one (a tenth of the set slots)."""
    k = np.where(has_mp != 0, 0, -1).astype(np.int32)
    k[(k == 0) & (rng.random(len(k)) < 0.1)] = 1
    return k


@pytest.mark.parametrize("ratio,ori", [(0.7, True), (0.6, False)])
def test_shim_search_by_bow(shim, tmp_path, ratio, ori):
    k1, k2, fv1, fv2 = _bow()
    a1, a2 = O.featvec_arrays(fv1), O.featvec_arrays(fv2)
    rng = np.random.default_rng(5)
    s1, s2 = _slot_kinds(k1["has_mp"], rng), _slot_kinds(k2["has_mp"], rng)
    cam = np.array([500, 500, 320, 240, 40], F32)
    kfa1 = _kf_arrays(k1, np.eye(4, dtype=F32), np.zeros(3, F32), cam, SF, ISG2, SG2, a1)
    kfa2 = _kf_arrays(k2, np.eye(4, dtype=F32), np.zeros(3, F32), cam, SF, ISG2, SG2, a2)
    par = np.array([ratio, 1.0 if ori else 0.0], F32)
    # keyframe-frame: the frame side is keyframe 2's features (no map-point condition there)
    fr = (np.asarray(k2["x"], F32), np.asarray(k2["y"], F32), np.asarray(k2["angle"], F32),
          np.asarray(k2["octave"], np.int32), np.ascontiguousarray(k2["desc"], np.uint8))
    r, outp = _run(shim, "sbbf", tmp_path, *kfa1, s1, *fr, *a2, par)
    assert r.returncode == 0, r.stderr
    n, mf = _read(outp, np.int32, np.int32)
    rn, rf = O.search_by_bow_frame(k1, (s1 == 0).astype(np.uint8), a1, k2, a2, ratio, ori)
    assert int(n[0]) == rn and np.array_equal(mf, rf) and rn > 50
    r, outp = _run(shim, "sbbk", tmp_path, *kfa1, s1, *kfa2, s2, par)
    assert r.returncode == 0, r.stderr
    n, m12 = _read(outp, np.int32, np.int32)
    rn, r12 = O.search_by_bow_kf(k1, (s1 == 0).astype(np.uint8), a1, k2, (s2 == 0).astype(np.uint8), a2, ratio, ori)
    assert int(n[0]) == rn and np.array_equal(m12, r12) and rn > 50


# ------------------------------------------------------------------ the threading contract
def test_shim_threading_contract(shim, tmp_path, amd):
    """handles are not reentrant but two extractor handles must run concurrently from
    two host threads (stereo L/R), and matcher / optimizer calls arrive from the Tracking and
    LocalMapping threads at once.  Five host threads start together and repeat their call: the
    stereo Frame (two more threads inside, one per extractor), SearchForInitialization,
    PoseOptimization, LocalBundleAdjustment and a second stereo Frame at another geometry.  Every
    repetition must be byte-identical to the first (no cross-thread interference) and the first
    must pass the same oracle checks as the single-threaded tests."""
    import subprocess
    from orb_slam2_amd import synth
    # stereo jobs
    st_a, imgs_a = _stereo_inputs(752, 480, 1200, 0x5EED0005, 4, EUROC_BF)
    st_b, imgs_b = _stereo_inputs(1241, 376, 2000, 0x5EED0003, 1, KITTI_BF)
    _write(tmp_path / "st_a.in", *st_a)
    _write(tmp_path / "st_b.in", *st_b)
    # SearchForInitialization job
    cv = synth.canvas(0x5EED0002, 640, 480)
    p = O.params(1000)
    a, b = O.extract(p, synth.frame(cv, 640, 480, 5)), O.extract(p, synth.frame(cv, 640, 480, 6))
    prev = np.stack([a["kps"]["x"], a["kps"]["y"]], 1).astype(F32).reshape(-1)
    _write(tmp_path / "sfi.in", *_frame_arrays(a["kps"], a["desc"]), *_frame_arrays(b["kps"], b["desc"]), GRID, prev,
           np.array([100], np.int32))
    # PoseOptimization job
    frame = synth.pose_problems(n_frames=1, stereo_frac=0.3, seed=21)[0]
    frame = dict(frame, cam=tuple(float(np.float32(v)) for v in frame["cam"]))
    pose_in, pos = _pose_inputs(frame, 8)
    _write(tmp_path / "pose.in", *pose_in)
    # LocalBundleAdjustment job (the layout of test_cpp_shim.test_shim_local_bundle_adjustment)
    pb = synth.ba_problem(n_local=8, n_fixed=3, n_points=900, stereo_frac=0.3, seed=11)
    octave = np.array([int(np.argmin(np.abs(INV_SIGMA2.astype(np.float64) - i))) for i in pb["edge_info"]], np.int32)
    _write(tmp_path / "lba.in", np.asarray(pb["Tcw"], F32).reshape(-1), np.asarray(pb["pose_fixed"], np.uint8),
           np.asarray(pb["pose_id"], np.int64), np.asarray(pb["point_xyz"], F32).reshape(-1),
           np.asarray(pb["point_id"], np.int64), np.asarray(pb["edge_point"], np.int32),
           np.asarray(pb["edge_pose"], np.int32), np.asarray(pb["edge_obs"], F32).reshape(-1), octave,
           np.asarray(pb["edge_cam"][0], F32), INV_SIGMA2, np.zeros(1, np.uint8))
    # fresh:pose — every PoseOptimization repetition on a new host thread, so its per-thread scratch
    # (stream + device buffer) is created while the LocalMapping job may be capturing its LM graph
    # (the creation takes the capture lock, common.h host_scratch)
    jobs = [("stereo", "st_a.in"), ("sfi", "sfi.in"), ("pose", "pose.in"), ("lba", "lba.in"), ("stereo", "st_b.in"),
            ("fresh:pose", "pose.in")]
    out = tmp_path / "thr.out"
    argv = [str(shim), "threads", str(out), "6"] + [x for m, f in jobs for x in (m, str(tmp_path / f))]
    r = subprocess.run(argv, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stderr)
    _check_stereo(f"{out}.0", imgs_a, 1200, EUROC_BF)
    _check_stereo(f"{out}.4", imgs_b, 2000, KITTI_BF)
    n, m12, _, _ = _read(f"{out}.1", np.int32, np.int32, F32, np.int32)
    fa, fb = O.FrameView(a["kps"], a["desc"], 640, 480), O.FrameView(b["kps"], b["desc"], 640, 480)
    n_ref, m_ref, _ = O.search_for_initialization(fa, fb, prev.copy(), nnratio=0.9, window=100)
    assert int(n[0]) == n_ref and np.array_equal(m12, m_ref)
    n, outl, T = _read(f"{out}.2", np.int32, np.uint8, F32)
    ref = O.pose_optimization(frame)
    assert int(n[0]) == ref["n_inliers"] and np.array_equal(outl[pos], ref["outlier"])
    assert (tmp_path / "thr.out.5").read_bytes() == (tmp_path / "thr.out.2").read_bytes()   # fresh-thread scratch
    res = _read(f"{out}.3", np.float64, np.float64, np.uint8, np.int64, np.float64, np.int64, np.uint8, np.int32,
                np.int32, np.uint8, np.float64, np.float64, np.float64, np.uint8, np.float64, np.float64, np.float64,
                np.int32)
    pq, pt, pfix, pid, X, xid, xbad, ept, eps, est, eobs, einfo, ecam, erase, oq, ot, ox, stt = res
    kf_of_pose = {int(i): k for k, i in enumerate(np.asarray(pb["pose_id"]))}
    Tcw = np.stack([np.asarray(pb["Tcw"], F32)[kf_of_pose[int(i)]] for i in pid])
    prob = dict(Tcw=Tcw, pose_fixed=pfix, pose_id=pid, point_xyz=X.reshape(-1, 3), point_id=xid, point_bad=xbad,
                edge_point=ept, edge_pose=eps, edge_stereo=est, edge_obs=eobs.reshape(-1, 3), edge_info=einfo,
                edge_cam=ecam.reshape(-1, 5))
    orc = O.lba_solve(prob)
    assert tuple(stt[:2]) == orc["iterations"] and int(stt[2]) == orc["trials"]
    assert np.array_equal(erase, orc["edge_erase"])
    assert np.abs(oq.reshape(-1, 4) - orc["pose_q"]).max() < 1e-5 and np.abs(ox.reshape(-1, 3) - orc["point_xyz"]).max() < 1e-5
