"""world_size-2 gloo tests of the multi-GPU algorithms on the CPU:
  * local BA with landmarks sharded over ranks and S / b_s / chi2 / scale all-reduced
    (the algorithm liborbslam2_amd runs over RCCL), restated in the oracle, must reproduce
    the single-process result (same LM decisions, 1e-9);
  * frame sharding for extraction: independent shards + max-over-ranks timing."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _lba_worker(rank, world, port, q):
    import sys
    import pathlib
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "tests")]
    import pkgload
    pkgload.load()
    from orb_slam2_amd import synth
    import oracle_ref as O
    _init(rank, world, port)
    pb = synth.ba_problem(n_points=1200, seed=21, stereo_frac=0.3)
    AR = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(C.c_double), C.c_int, C.c_int)

    def ar(user, ptr, n, op):
        a = np.ctypeslib.as_array(ptr, shape=(n,))
        t = torch.from_numpy(a)
        dist.all_reduce(t, op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MAX)

    cb = AR(ar)
    lib = O.lib()
    lib.oracle_lba_solve_dist.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, AR,
                                          C.c_void_p]
    nk = len(pb["Tcw"])
    qs, ts = zip(*[O.quat_from_Tcw(T) for T in pb["Tcw"]])
    qa, ta = np.ascontiguousarray(qs), np.ascontiguousarray(ts)
    a = {k: np.ascontiguousarray(v) for k, v in pb.items()}
    P = O.P
    pr = O.LbaProblem(nk, P(qa), P(ta), P(a["pose_fixed"]), P(a["pose_id"]), len(a["point_xyz"]), P(a["point_xyz"]),
                      P(a["point_id"]), P(a["point_bad"]), len(a["edge_point"]), P(a["edge_point"]),
                      P(a["edge_pose"]), P(a["edge_stereo"]), P(a["edge_obs"]), P(a["edge_info"]), P(a["edge_cam"]))
    out = dict(pose_q=np.zeros((nk, 4)), pose_t=np.zeros((nk, 3)), point_xyz=np.zeros_like(a["point_xyz"]),
               edge_erase=np.zeros(len(a["edge_point"]), np.uint8), trace=np.zeros((64, 4)))
    r = O.LbaResult(P(out["pose_q"]), P(out["pose_t"]), P(out["point_xyz"]), P(out["edge_erase"]), None,
                    (C.c_int * 2)(0, 0), 0, P(out["trace"]), 0)
    opts = O.lba_options()
    flag = (C.c_uint8 * 1)(0)
    lib.oracle_lba_solve_dist(C.byref(pr), C.byref(opts), flag, C.byref(r), rank, world, cb, None)
    ref = O.lba_solve(pb) if rank == 0 else None
    M = len(a["point_xyz"])
    own = slice(M * rank // world, M * (rank + 1) // world)
    res = dict(iterations=tuple(r.iterations), trials=r.trials, trace=out["trace"][: r.n_trace].copy(),
               pose_q=out["pose_q"], pose_t=out["pose_t"], own=(own.start, own.stop),
               points=out["point_xyz"][own].copy(), erase=out["edge_erase"].copy())
    q.put((rank, res, ref))
    dist.destroy_process_group()


def test_sharded_local_ba_matches_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lba_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        rank, res, ref = q.get(timeout=300)
        results[rank] = (res, ref)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = results[0][1]
    erase = np.zeros_like(ref["edge_erase"])
    for rank in range(world):
        res = results[rank][0]
        assert res["iterations"] == ref["iterations"] and res["trials"] == ref["trials"]
        assert np.allclose(res["trace"][:, :3], ref["trace"][:, :3], rtol=1e-9)
        assert np.abs(res["pose_q"] - ref["pose_q"]).max() < 1e-9
        assert np.abs(res["pose_t"] - ref["pose_t"]).max() < 1e-9
        a, b = res["own"]
        assert np.abs(res["points"] - ref["point_xyz"][a:b]).max() < 1e-9
        erase |= res["erase"]
    assert np.array_equal(erase, ref["edge_erase"])


def _frames_worker(rank, world, port, q):
    import sys
    import pathlib
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "tests")]
    import time
    import pkgload
    pkgload.load()
    from orb_slam2_amd import synth
    import oracle_ref as O
    _init(rank, world, port)
    cv = synth.canvas(0x5EED0002 + 1000 * rank, 640, 480)     # bench.py: independent stream per rank
    t0 = time.perf_counter()
    n = [len(O.extract(O.params(1000), synth.frame(cv, 640, 480, t))["kps"]) for t in range(2)]
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.barrier()
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    tot = torch.tensor([float(sum(n))], dtype=torch.float64)
    dist.all_reduce(tot)
    q.put((rank, float(dt.item()), float(tot.item()), n))
    dist.destroy_process_group()


def test_frame_sharding_weak_scaling():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_frames_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dts = {o[1] for o in out}
    assert len(dts) == 1                       # every rank sees the same max time
    assert out[0][2] == sum(sum(o[3]) for o in out)
