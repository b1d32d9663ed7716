"""Runs a few LocalBundleAdjustment solves of the config-4 problem (corridor=1 n_local=200
n_points=100000: the scaled window; group=N: through lba_group on N contexts of device 0, with the
per-collective exchange time of the group's all-reduce) and prints
per-stage event times; with ORB_SLAM2_AMD_LIB pointing at an ORB_TIMING variant
(tools/build_variant.py timing -DORB_TIMING) the kernels print their own clock splits."""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import pkgload  # noqa: E402

amd = pkgload.load()
from orb_slam2_amd import synth  # noqa: E402

kw = {}
for a in sys.argv[1:]:
    k, v = a.split("=")
    kw[k] = float(v) if "." in v else int(v)
# corridor=1: the scaled window generator (synth.ba_problem_corridor, banded covisibility)
gen = synth.ba_problem_corridor if kw.pop("corridor", 0) else synth.ba_problem
group = kw.pop("group", 0)
n = kw.pop("solves", 12)   # (under rocprofv3's kernel trace, 200 KF runs keep to a few solves)
pb = gen(**kw)
print(f"problem: {len(pb['Tcw'])} keyframes, {len(pb['point_xyz'])} points, {len(pb['edge_point'])} edges", flush=True)
ba = amd.LocalBAGroup([0] * group) if group else amd.LocalBA()
call = ba.prepared(pb)
ts = []
for i in range(n):
    t0 = time.perf_counter()
    its, trials, _ = call()
    dt = time.perf_counter() - t0
    ts.append(dt)
    print(f"solve {i}: {dt * 1e3:.3f} ms, iterations {its}, trials {trials}", flush=True)
    if group and i == 3:
        ex0 = ba.stats()
import statistics  # noqa: E402
print(f"median of solves {min(4, n - 1)}..{n - 1}: {1e3 * statistics.median(ts[min(4, n - 1):]):.3f} ms", flush=True)
if group:
    ex1 = ba.stats()
    nc = ex1[1] - ex0[1]
    if ex1[0] > 0:
        print(f"group of {group}: {nc} collectives in solves 4..{n - 1}, exchange {1e3 * (ex1[0] - ex0[0]) / max(nc, 1):.2f} us "
              f"per collective (rank 0's stream, events around the all-reduce)", flush=True)
    else:
        print(f"group of {group}: {nc} collectives in solves 4..{n - 1} (device-side exchange: per-collective time "
              f"from the kernel trace, k_grp_sync / k_grp_reduce)", flush=True)
