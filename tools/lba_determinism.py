"""Diagnostic: is the GPU local BA bitwise reproducible across solves and contexts?  Compares the
final LM state's buffers (lba_debug_buffer) of repeated one-iteration solves."""
import sys
import pathlib
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import numpy as np
import pkgload
amd = pkgload.load()
from orb_slam2_amd import synth, optimizer

pb = synth.ba_problem(n_points=300, seed=6)
names = ["S", "bs", "x", "Hpp", "bp", "Hll", "bl", "Dinv"]
ctx = amd.LocalBA()
o = optimizer.options(1, 0, fixed_iterations=True)
runs = []
for _ in range(6):
    ctx.solve(pb, o)
    runs.append([ctx.debug_buffer(i) for i in range(8)])
for i, nm in enumerate(names):
    print(nm, [float(np.abs(r[i] - runs[0][i]).max()) for r in runs])
S = runs[0][0]
n = int(round(np.sqrt(len(S))))
S = S.reshape(n, n)
print("S symmetric", float(np.abs(S - S.T).max()), "n", n)
for r in runs:
    xs = ctx.dense_solve(r[0].reshape(n, n), r[1])
    print("dense_solve vs x", float(np.abs(xs - r[2][:n]).max()))
