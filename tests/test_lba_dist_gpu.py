"""The library's multi-GPU local BA path (landmark shards + all-reduce callback),
rehearsed with 2 processes on one GPU over gloo: identical to the single-GPU run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    import pathlib
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "tests")]
    import torch.distributed as dist
    import pkgload
    amd = pkgload.load()
    from orb_slam2_amd import synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())   # explicit stream shared by torch and the solver
    pb = synth.ba_problem(n_points=2000, seed=13, stereo_frac=0.25)
    nk, ne = len(pb["Tcw"]), len(pb["edge_point"])
    ws = torch.zeros(max(36 * nk * nk + 6 * nk, ne) + 64, dtype=torch.float64, device="cuda")

    def ar(off, cnt, op):
        dist.all_reduce(ws[off:off + cnt], op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MAX)

    ctx = amd.LocalBA(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.set_comm(rank, world, ws, ar)
    res = ctx.solve(pb)
    ref = amd.LocalBA(0).solve(pb) if rank == 0 else None
    M = len(pb["point_xyz"])
    a, b = M * rank // world, M * (rank + 1) // world
    q.put((rank, dict(iterations=res["iterations"], trials=res["trials"], trace=res["trace"], pose_q=res["pose_q"],
                      pose_t=res["pose_t"], own=(a, b), points=res["point_xyz"][a:b], erase=res["edge_erase"]), ref))
    dist.destroy_process_group()


def test_two_rank_local_ba_matches_single_gpu():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, res, ref = q.get(timeout=300)
        out[rank] = (res, ref)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = out[0][1]
    erase = np.zeros_like(ref["edge_erase"])
    for rank in range(world):
        res = out[rank][0]
        assert res["iterations"] == ref["iterations"] and res["trials"] == ref["trials"]
        assert np.allclose(res["trace"][:, :3], ref["trace"][:, :3], rtol=1e-9)
        assert np.abs(res["pose_q"] - ref["pose_q"]).max() < 1e-9
        a, b = res["own"]
        assert np.abs(res["points"] - ref["point_xyz"][a:b]).max() < 1e-9
        erase |= res["erase"]
    assert np.array_equal(erase, ref["edge_erase"])
