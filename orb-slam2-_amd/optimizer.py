"""Host mirror of ORB_SLAM2::Optimizer::LocalBundleAdjustment
(R/include/Optimizer.h:45, R/src/Optimizer.cpp:564-918) and Optimizer::PoseOptimization
(R/include/Optimizer.h:44, R/src/Optimizer.cpp:306-535) over the HIP C-ABI.

The graph-gathering part of the reference (local / fixed keyframes, local map
points, edge construction, R :569-782) is host bookkeeping on Map/KeyFrame/
MapPoint objects; callers pass the resulting graph as arrays (see
synth.ba_problem for the layout).  lba_solve runs the optimisation and the
outlier passes on the GPU; apply_results mirrors the write-back (R :883-917)."""
import ctypes as C

import numpy as np

from . import _abi


class LbaProblem(C.Structure):
    _fields_ = [("n_poses", C.c_int), ("pose_q", C.c_void_p), ("pose_t", C.c_void_p), ("pose_fixed", C.c_void_p),
                ("pose_id", C.c_void_p), ("n_points", C.c_int), ("point_xyz", C.c_void_p), ("point_id", C.c_void_p),
                ("point_bad", C.c_void_p), ("n_edges", C.c_int), ("edge_point", C.c_void_p),
                ("edge_pose", C.c_void_p), ("edge_stereo", C.c_void_p), ("edge_obs", C.c_void_p),
                ("edge_info", C.c_void_p), ("edge_cam", C.c_void_p)]


class LbaOptions(C.Structure):
    _fields_ = [("iters1", C.c_int), ("iters2", C.c_int), ("chi2_mono", C.c_double), ("chi2_stereo", C.c_double),
                ("huber_mono", C.c_double), ("huber_stereo", C.c_double), ("max_trials", C.c_int),
                ("fixed_iterations", C.c_int)]


class LbaResult(C.Structure):
    _fields_ = [("pose_q", C.c_void_p), ("pose_t", C.c_void_p), ("point_xyz", C.c_void_p),
                ("edge_erase", C.c_void_p), ("edge_chi2", C.c_void_p), ("iterations", C.c_int * 2),
                ("trials", C.c_int), ("trace", C.c_void_p), ("n_trace", C.c_int), ("aborted", C.c_int)]


# lba_problem's field types (include/orbslam2_amd.h); Tcw is converted separately
PROBLEM_DTYPES = {"pose_fixed": np.uint8, "pose_id": np.int64, "point_xyz": np.float64, "point_id": np.int64,
                  "point_bad": np.uint8, "edge_point": np.int32, "edge_pose": np.int32, "edge_stereo": np.uint8,
                  "edge_obs": np.float64, "edge_info": np.float64, "edge_cam": np.float64}

ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_size_t, C.c_size_t, C.c_int)


def options(iters1=5, iters2=10, fixed_iterations=False):
    """Constants of R/src/Optimizer.cpp:696-697, 790, 814, 841 and g2o's maxTrialsAfterFailure."""
    return LbaOptions(iters1, iters2, 5.991, 7.815, float(np.float32(np.sqrt(5.991))),
                      float(np.float32(np.sqrt(7.815))), 10, int(fixed_iterations))


def global_options(nIterations=10, fixed_iterations=False):
    """Optimizer::BundleAdjustment's constants (R/src/Optimizer.cpp:117-118): thHuber2D =
    (float)sqrt(5.99), thHuber3D = (float)sqrt(7.815); nIterations in iters1."""
    return LbaOptions(nIterations, 0, 5.991, 7.815, float(np.float32(np.sqrt(5.99))),
                      float(np.float32(np.sqrt(7.815))), 10, int(fixed_iterations))


def _sig():
    lib = _abi.lib()
    if getattr(lib, "_lba_sig", False):
        return lib
    vp, i32, sz = C.c_void_p, C.c_int, C.c_size_t
    for name, args, res in [("lba_create", [i32, vp], C.c_int), ("lba_destroy", [vp], None),
                            ("lba_set_stream", [vp, vp, i32], C.c_int),
                            ("lba_set_comm", [vp, i32, i32, vp, sz, ALLREDUCE_FN, vp], C.c_int),
                            ("lba_solve", [vp, vp, vp, vp, vp], C.c_int), ("lba_profile", [vp, i32], C.c_int),
                            ("lba_solve_global", [vp, vp, vp, i32, vp, vp], C.c_int),
                            ("lba_stats", [vp, vp, vp, vp], C.c_int),
                            ("lba_debug_stop_after_trials", [vp, i32], C.c_int),
                            ("lba_debug_buffer", [vp, i32, vp, sz], C.c_int),
                            ("lba_dense_solve", [vp, vp, vp, i32, vp], C.c_int), ("lba_pose_from_Tcw", [vp, vp, vp], None),
                            ("lba_pose_to_Tcw", [vp, vp, vp], None),
                            ("lba_poses_from_Tcw", [vp, i32, vp, vp], None),
                            ("lba_group_create", [vp, i32, vp], C.c_int), ("lba_group_destroy", [vp], None),
                            ("lba_group_solve", [vp, vp, vp, vp, vp], C.c_int),
                            ("lba_group_stats", [vp, vp, vp], C.c_int)]:
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    lib._lba_sig = True
    return lib


def pose_from_Tcw(T):
    """Converter::toSE3Quat on a float Tcw."""
    T = np.ascontiguousarray(np.asarray(T, np.float32).reshape(4, 4))
    q, t = np.zeros(4), np.zeros(3)
    _sig().lba_pose_from_Tcw(_abi.ptr(T), _abi.ptr(q), _abi.ptr(t))
    return q, t


def pose_to_Tcw(q, t):
    """Converter::toCvMat(SE3Quat) (float 4x4)."""
    T = np.zeros((4, 4), np.float32)
    _sig().lba_pose_to_Tcw(_abi.ptr(np.ascontiguousarray(q, np.float64)), _abi.ptr(np.ascontiguousarray(t, np.float64)),
                           _abi.ptr(T))
    return T


class LocalBA:
    """A reusable GPU context (one HIP stream) for LocalBundleAdjustment."""

    def __init__(self, device=0):
        h = C.c_void_p()
        _abi.check("lba_create", _sig().lba_create(device, C.byref(h)))
        self._h = h
        self._comm = None

    def close(self):
        if getattr(self, "_h", None):
            _sig().lba_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def set_stream(self, stream_handle):
        """Run on the given hipStream_t handle (e.g. torch.cuda.current_stream().cuda_stream;
        0 = the legacy default stream) so torch collectives are ordered with the solver."""
        _abi.check("lba_set_stream", _sig().lba_set_stream(self._h, C.c_void_p(stream_handle or 0), 1))

    def set_comm(self, rank, world, workspace, allreduce):
        """workspace: a float64 device tensor; allreduce(offset, count, op) reduces a slice of it."""
        def cb(user, offset, count, op):
            try:
                allreduce(int(offset), int(count), int(op))
                return 0
            except Exception as exc:  # noqa: BLE001 - reported through the C status
                print(f"lba allreduce failed: {exc}")
                return 1
        self._comm = (ALLREDUCE_FN(cb), workspace)
        _abi.check("lba_set_comm", _sig().lba_set_comm(self._h, rank, world, C.c_void_p(workspace.data_ptr()),
                                                        workspace.numel(), self._comm[0], None))

    def dense_solve(self, S, b):
        """x = S^-1 b through the reduced-camera-system LDL^T (lba_dense_solve)."""
        S = np.ascontiguousarray(S, dtype=np.float64)
        b = np.ascontiguousarray(b, dtype=np.float64)
        x = np.zeros(len(b))
        _abi.check("lba_dense_solve", _sig().lba_dense_solve(self._h, _abi.ptr(S), _abi.ptr(b), len(b), _abi.ptr(x)))
        return x

    def profile(self, enable=True):
        _sig().lba_profile(self._h, int(enable))

    def debug_buffer(self, which):
        """A device buffer of the last solve (lba_debug_buffer: 0 S, 1 b_s, 2 x, 3 Hpp, 4 b_p, 5 Hll,
        6 b_l, 7 D^-1) as a float64 array."""
        n = _sig().lba_debug_buffer(self._h, which, _abi.ptr(np.zeros(1)), 0)
        _abi.check("lba_debug_buffer", n)
        out = np.zeros(n)
        _abi.check("lba_debug_buffer", _sig().lba_debug_buffer(self._h, which, _abi.ptr(out), n))
        return out

    def debug_stop_after_trials(self, n):
        """Test hook: behave as if the stop flag became set when the solve's trial count reached n
        (None / negative: off)."""
        _abi.check("lba_debug_stop_after_trials",
                   _sig().lba_debug_stop_after_trials(self._h, -1 if n is None else int(n)))

    def stats(self):
        ms = np.zeros(4)
        it, tr = C.c_int(), C.c_int()
        _sig().lba_stats(self._h, _abi.ptr(ms), C.byref(it), C.byref(tr))
        return dict(linearize_ms=ms[0], schur_ms=ms[1], solve_ms=ms[2], update_ms=ms[3], iterations=it.value,
                    trials=tr.value)

    def prepared(self, prob, opts=None):
        """The lba_solve call of solve(prob) with its arguments marshalled once: returns a
        zero-argument callable that runs only the C-ABI call (the benchmark's timed region) and
        returns (iterations, trials)."""
        opts = opts or options()
        nk = len(prob["Tcw"])
        Tcw = np.ascontiguousarray(prob["Tcw"], np.float32)
        q, t = np.zeros((nk, 4)), np.zeros((nk, 3))
        _sig().lba_poses_from_Tcw(_abi.ptr(Tcw), nk, _abi.ptr(q), _abi.ptr(t))
        a = {k: np.ascontiguousarray(v, PROBLEM_DTYPES[k]) if k in PROBLEM_DTYPES and v is not None else v
             for k, v in prob.items()}
        P = _abi.ptr
        pr = LbaProblem(nk, P(q), P(t), P(a["pose_fixed"]), P(a["pose_id"]), len(a["point_xyz"]), P(a["point_xyz"]),
                        P(a["point_id"]), P(a.get("point_bad")), len(a["edge_point"]), P(a["edge_point"]),
                        P(a["edge_pose"]), P(a["edge_stereo"]), P(a["edge_obs"]), P(a["edge_info"]), P(a["edge_cam"]))
        ne = len(a["edge_point"])
        out = dict(pose_q=np.zeros((nk, 4)), pose_t=np.zeros((nk, 3)), point_xyz=a["point_xyz"].copy(),
                   edge_erase=np.zeros(ne, np.uint8), edge_chi2=np.zeros(ne), trace=np.zeros((64, 4)))
        r = LbaResult(P(out["pose_q"]), P(out["pose_t"]), P(out["point_xyz"]), P(out["edge_erase"]),
                      P(out["edge_chi2"]), (C.c_int * 2)(0, 0), 0, P(out["trace"]), 0, 0)
        flag = (C.c_uint8 * 1)(0)
        keep = (q, t, a, out, Tcw)   # the arrays the structs point into stay alive with the closure
        fn, h, rp, op, rr = _sig().lba_solve, self._h, C.byref(pr), C.byref(opts), C.byref(r)

        def call():
            _abi.check("lba_solve", fn(h, rp, op, flag, rr))
            return (r.iterations[0], r.iterations[1]), r.trials, keep
        return call

    def solve(self, prob, opts=None, stop=None, global_ba=False, robust=True):
        """prob: dict of arrays (synth.ba_problem layout).  stop: a 1-byte ctypes array
        polled like mbAbortBA.  global_ba: Optimizer::BundleAdjustment instead of the local BA
        flow (lba_solve_global; opts from global_options, robust = bRobust).  Returns a dict
        with the optimised estimates."""
        opts = opts or (global_options() if global_ba else options())
        nk = len(prob["Tcw"])
        Tcw = np.ascontiguousarray(prob["Tcw"], np.float32)
        q, t = np.zeros((nk, 4)), np.zeros((nk, 3))
        _sig().lba_poses_from_Tcw(_abi.ptr(Tcw), nk, _abi.ptr(q), _abi.ptr(t))   # Converter::toSE3Quat
        # each field coerced to the C type lba_problem declares (include/orbslam2_amd.h)
        a = {k: np.ascontiguousarray(v, PROBLEM_DTYPES[k]) if k in PROBLEM_DTYPES and v is not None else v
             for k, v in prob.items()}
        P = _abi.ptr
        pr = LbaProblem(nk, P(q), P(t), P(a["pose_fixed"]), P(a["pose_id"]), len(a["point_xyz"]), P(a["point_xyz"]),
                        P(a["point_id"]), P(a.get("point_bad")), len(a["edge_point"]), P(a["edge_point"]),
                        P(a["edge_pose"]), P(a["edge_stereo"]), P(a["edge_obs"]), P(a["edge_info"]), P(a["edge_cam"]))
        ne = len(a["edge_point"])
        out = dict(pose_q=np.zeros((nk, 4)), pose_t=np.zeros((nk, 3)), point_xyz=a["point_xyz"].copy(),
                   edge_erase=np.zeros(ne, np.uint8), edge_chi2=np.zeros(ne), trace=np.zeros((64, 4)))
        r = LbaResult(P(out["pose_q"]), P(out["pose_t"]), P(out["point_xyz"]), P(out["edge_erase"]),
                      P(out["edge_chi2"]), (C.c_int * 2)(0, 0), 0, P(out["trace"]), 0, 0)
        flag = stop if stop is not None else (C.c_uint8 * 1)(0)
        if global_ba:
            _abi.check("lba_solve_global", _sig().lba_solve_global(self._h, C.byref(pr), C.byref(opts), int(robust), flag,
                                                                    C.byref(r)))
        else:
            _abi.check("lba_solve", _sig().lba_solve(self._h, C.byref(pr), C.byref(opts), flag, C.byref(r)))
        out["iterations"] = (r.iterations[0], r.iterations[1])
        out["trials"] = r.trials
        out["trace"] = out["trace"][: r.n_trace]
        out["aborted"] = bool(r.aborted)
        out["init_q"], out["init_t"] = q, t
        return out


def _marshal(prob):
    """lba_problem / lba_result structs over numpy copies of `prob` (kept alive in the tuple)."""
    nk = len(prob["Tcw"])
    Tcw = np.ascontiguousarray(prob["Tcw"], np.float32)
    q, t = np.zeros((nk, 4)), np.zeros((nk, 3))
    _sig().lba_poses_from_Tcw(_abi.ptr(Tcw), nk, _abi.ptr(q), _abi.ptr(t))   # Converter::toSE3Quat
    a = {k: np.ascontiguousarray(v, PROBLEM_DTYPES[k]) if k in PROBLEM_DTYPES and v is not None else v
         for k, v in prob.items()}
    P = _abi.ptr
    pr = LbaProblem(nk, P(q), P(t), P(a["pose_fixed"]), P(a["pose_id"]), len(a["point_xyz"]), P(a["point_xyz"]),
                    P(a["point_id"]), P(a.get("point_bad")), len(a["edge_point"]), P(a["edge_point"]),
                    P(a["edge_pose"]), P(a["edge_stereo"]), P(a["edge_obs"]), P(a["edge_info"]), P(a["edge_cam"]))
    ne = len(a["edge_point"])
    out = dict(pose_q=np.zeros((nk, 4)), pose_t=np.zeros((nk, 3)), point_xyz=a["point_xyz"].copy(),
               edge_erase=np.zeros(ne, np.uint8), edge_chi2=np.zeros(ne), trace=np.zeros((64, 4)))
    r = LbaResult(P(out["pose_q"]), P(out["pose_t"]), P(out["point_xyz"]), P(out["edge_erase"]),
                  P(out["edge_chi2"]), (C.c_int * 2)(0, 0), 0, P(out["trace"]), 0, 0)
    return pr, r, out, (q, t, a, Tcw)


class LocalBAGroup:
    """Multi-GPU LocalBundleAdjustment from one process (lba_group_*): one context per entry of
    `devices` (a device may repeat), landmarks sharded over them, the reduced system all-reduced
    by the library's peer-to-peer kernel over xGMI."""

    def __init__(self, devices):
        devs = (C.c_int * len(devices))(*[int(d) for d in devices])
        h = C.c_void_p()
        _abi.check("lba_group_create", _sig().lba_group_create(devs, len(devices), C.byref(h)))
        self._h = h
        self.devices = list(devices)

    def close(self):
        if getattr(self, "_h", None):
            _sig().lba_group_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def prepared(self, prob, opts=None):
        opts = opts or options()
        pr, r, out, keep = _marshal(prob)
        flag = (C.c_uint8 * 1)(0)
        fn, h = _sig().lba_group_solve, self._h

        def call():
            _abi.check("lba_group_solve", fn(h, C.byref(pr), C.byref(opts), flag, C.byref(r)))
            return (r.iterations[0], r.iterations[1]), r.trials, (keep, out)
        return call

    def solve(self, prob, opts=None, stop=None):
        opts = opts or options()
        pr, r, out, keep = _marshal(prob)
        flag = stop if stop is not None else (C.c_uint8 * 1)(0)
        _abi.check("lba_group_solve", _sig().lba_group_solve(self._h, C.byref(pr), C.byref(opts), flag, C.byref(r)))
        out["iterations"] = (r.iterations[0], r.iterations[1])
        out["trials"] = r.trials
        out["trace"] = out["trace"][: r.n_trace]
        out["aborted"] = bool(r.aborted)
        out["init_q"], out["init_t"] = keep[0], keep[1]
        return out

    def stats(self):
        """(total exchange ms on rank 0's stream, number of collectives) since creation."""
        ms, n = C.c_double(), C.c_long()
        _abi.check("lba_group_stats", _sig().lba_group_stats(self._h, C.byref(ms), C.byref(n)))
        return ms.value, n.value


class Optimizer:
    """Namespace mirroring ORB_SLAM2::Optimizer's static interface for this path."""

    _ctx = {}

    @staticmethod
    def PoseOptimization(frames, device=0):
        """Batched Optimizer::PoseOptimization (see the module-level PoseOptimization)."""
        return PoseOptimization(frames, device)

    @staticmethod
    def LocalBundleAdjustment(problem, pbStopFlag=None, device=0, opts=None):
        ctx = Optimizer._ctx.get(device)
        if ctx is None:
            ctx = Optimizer._ctx[device] = LocalBA(device)
        return ctx.solve(problem, opts, pbStopFlag)

    @staticmethod
    def BundleAdjustment(problem, nIterations=5, pbStopFlag=None, bRobust=True, device=0, fixed_iterations=False):
        """Optimizer::BundleAdjustment (R/src/Optimizer.cpp:78-277) on the array form: every
        keyframe pose (pose_fixed = mnId == 0) and map point of `problem`; GlobalBundleAdjustemnt
        passes nIterations 20 (initialisation) or 10 (loop closing) and bRobust false there."""
        ctx = Optimizer._ctx.get(device)
        if ctx is None:
            ctx = Optimizer._ctx[device] = LocalBA(device)
        return ctx.solve(problem, global_options(nIterations, fixed_iterations), pbStopFlag, global_ba=True,
                         robust=bRobust)


def apply_results(problem, result):
    """Write-back of R/src/Optimizer.cpp:883-917 on the array form: returns the
    (keyframe, point) observations to erase and float Tcw / world positions."""
    erase = [(int(problem["edge_pose"][e]), int(problem["edge_point"][e]))
             for e in np.nonzero(result["edge_erase"])[0]]
    Tcw = np.stack([pose_to_Tcw(q, t) for q, t in zip(result["pose_q"], result["pose_t"])])
    return erase, Tcw, result["point_xyz"].astype(np.float32)


class PoseBatch(C.Structure):
    _fields_ = [("n_frames", C.c_int), ("n_edges", C.c_int), ("pose_q", C.c_void_p), ("pose_t", C.c_void_p),
                ("cam", C.c_void_p), ("edge_start", C.c_void_p), ("edge_obs", C.c_void_p), ("edge_xw", C.c_void_p),
                ("edge_info", C.c_void_p)]


class PoseBatchResult(C.Structure):
    _fields_ = [("pose_q", C.c_void_p), ("pose_t", C.c_void_p), ("outlier", C.c_void_p), ("n_inliers", C.c_void_p)]


def _pose_sig():
    lib = _abi.lib()
    if not getattr(lib, "_pose_sig", False):
        _abi.sig(lib.pose_optimize_batch, [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p], C.c_int)
        _abi.sig(lib.pose_optimize_batch_device, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                   C.c_void_p], C.c_int)
        lib._pose_sig = True
    return lib


def pack_pose_frames(frames):
    """Frame dicts (synth.pose_problems layout: Tcw float 4x4, obs [n,3] with ur < 0 for mono,
    xw [n,3], info [n], cam (fx, fy, cx, cy, bf)) -> the flat arrays of pose_batch."""
    B = len(frames)
    Tcw = np.ascontiguousarray(np.stack([f["Tcw"] for f in frames]).astype(np.float32))
    q, t = np.zeros((B, 4)), np.zeros((B, 3))
    _sig().lba_poses_from_Tcw(_abi.ptr(Tcw), B, _abi.ptr(q), _abi.ptr(t))   # Converter::toSE3Quat
    counts = [len(f["info"]) for f in frames]
    start = np.zeros(B + 1, np.int32)
    start[1:] = np.cumsum(counts)
    cat = (lambda k: np.ascontiguousarray(np.concatenate([np.asarray(f[k], np.float64) for f in frames]))
           if B else np.zeros(0))
    return dict(pose_q=q, pose_t=t, cam=np.ascontiguousarray(np.array([f["cam"] for f in frames], np.float64)),
                edge_start=start, edge_obs=cat("obs").reshape(-1, 3), edge_xw=cat("xw").reshape(-1, 3),
                edge_info=cat("info"))


def PoseOptimization(frames, device=0):
    """ORB_SLAM2::Optimizer::PoseOptimization(Frame*) (R/src/Optimizer.cpp:306-535) over a batch
    of frames on the GPU.  Returns per frame the optimised pose (q, t as SE3Quat), mvbOutlier and
    the return value (nInitialCorrespondences - nBad), plus LM iterations per round / trials."""
    a = pack_pose_frames(frames)
    B, E = len(frames), int(a["edge_start"][-1])
    pb = PoseBatch(B, E, _abi.ptr(a["pose_q"]), _abi.ptr(a["pose_t"]), _abi.ptr(a["cam"]), _abi.ptr(a["edge_start"]),
                   _abi.ptr(a["edge_obs"]), _abi.ptr(a["edge_xw"]), _abi.ptr(a["edge_info"]))
    q, t = np.zeros((B, 4)), np.zeros((B, 3))
    outl, ninl, iters = np.zeros(E, np.uint8), np.zeros(B, np.int32), np.zeros((B, 5), np.int32)
    r = PoseBatchResult(_abi.ptr(q), _abi.ptr(t), _abi.ptr(outl), _abi.ptr(ninl))
    _abi.check("pose_optimize_batch", _pose_sig().pose_optimize_batch(device, C.byref(pb), C.byref(r),
                                                                        _abi.ptr(iters)))
    s = a["edge_start"]
    return [dict(pose_q=q[b], pose_t=t[b], outlier=outl[s[b]:s[b + 1]], n_inliers=int(ninl[b]),
                 iterations=tuple(int(x) for x in iters[b, :4]), trials=int(iters[b, 4])) for b in range(B)]
