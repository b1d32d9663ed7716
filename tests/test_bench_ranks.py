"""bench.py's multi-GPU launcher: `--gpus N` without a torch.distributed launcher spawns N ranks
(one process per GPU; on a one-GPU lease the ranks share the device and the collectives run over
gloo).  The line must report the world size the ranks saw, and the landmark-sharded local BA must
take the same LM decisions as one rank."""
import json
import os
import pathlib
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parents[1]
ARGS = ["--steps", "2", "--warmup", "1", "--batch", "8", "--streams", "1", "--pool", "16", "--no-cpu", "--no-lba-scaled",
        "--no-extras", "--no-profile", "--lba-solves", "1", "--lba-points", "1500", "--stereo-batches", "2"]


def _run(n, extra=(), timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), *ARGS, *extra], env=env,
                         capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_report_world_and_agree_with_one():
    one, two = _run(1), _run(2)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2 and two["world_size"] == 2
    assert two["value"] > 0
    d1, d2 = one["lba"]["decisions"], two["lba"]["decisions"]
    assert d1["iterations"] == d2["iterations"] and d1["trials"] == d2["trials"]
    assert d1["erased_edges"] == d2["erased_edges"]
    for a, b in zip(d1["chi2_trace"], d2["chi2_trace"]):
        assert abs(a - b) <= 1e-9 * abs(a)
    c1, c2 = one["config5_stereo_sharded"], two["config5_stereo_sharded"]
    for tag in ("throughput", "latency_one_batch"):
        assert c1[tag]["stereo_matches_per_pair"] == c2[tag]["stereo_matches_per_pair"]
        # mvuRight / mvDepth of every pair identical whether one rank or two computed it
        assert c1[tag]["uright_depth_sha16"] == c2[tag]["uright_depth_sha16"]
    # frame shards: both ranks' sequences carried no truncation
    assert one["status"] == {"extractor": 0, "matcher": 0} and two["status"] == {"extractor": 0, "matcher": 0}


def _agree(one, many):
    d1, d2 = one["lba"]["decisions"], many["lba"]["decisions"]
    assert d1["iterations"] == d2["iterations"] and d1["trials"] == d2["trials"]
    assert d1["erased_edges"] == d2["erased_edges"]
    for a, b in zip(d1["chi2_trace"], d2["chi2_trace"]):
        assert abs(a - b) <= 1e-9 * abs(a)
    for tag in ("throughput", "latency_one_batch"):
        assert one["config5_stereo_sharded"][tag]["uright_depth_sha16"] == \
            many["config5_stereo_sharded"][tag]["uright_depth_sha16"]


def test_bench_eight_ranks_rehearsal():
    """The driver's N = 8 launch rehearsed on one GPU: eight ranks (gloo, the device shared), one
    config-5 stereo pair each, landmarks of the local BA sharded eight ways over the default RCCL /
    torch.distributed callback — the same LM decisions and stereo digests as one rank."""
    one, eight = _run(1), _run(8, timeout=600)
    assert eight["n_gpus"] == 8 and eight["world_size"] == 8 and eight["value"] > 0
    assert eight["status"] == {"extractor": 0, "matcher": 0}
    assert eight["lba"]["collective"].startswith("torch.distributed")
    _agree(one, eight)


def test_bench_two_ranks_native_group():
    """--lba-comm native: rank 0 drives the library's device group over both ranks' devices
    (here one device: the host-ordered exchange) with the single-rank decisions."""
    one, two = _run(1), _run(2, ["--lba-comm", "native"])
    assert two["lba"]["native_group_unavailable"] is None and two["lba"]["collective"].startswith("library")
    _agree(one, two)
