"""Diagnostic: bitwise reproducibility of the reduced-system LDL^T (lba_dense_solve)."""
import sys
import pathlib
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import numpy as np
import pkgload
amd = pkgload.load()
for n in (60, 114, 120, 128, 200):
    rng = np.random.default_rng(n)
    G = rng.standard_normal((n, n + 8))
    S = G @ G.T + n * np.eye(n)
    b = rng.standard_normal(n)
    ctx = amd.LocalBA()
    xs = [ctx.dense_solve(S, b) for _ in range(20)]
    nd = sum(not np.array_equal(x, xs[0]) for x in xs)
    print(n, "differing runs:", nd, "max diff", max(np.abs(x - xs[0]).max() for x in xs))
