"""Repeated dense reduced-system solves (k_ldlt_solve alone, n = 114) so the kernel runs with a
warm instruction cache; with the ORB_TIMING variant the kernel prints its clock split."""
import pathlib
import sys

import numpy as np

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import pkgload  # noqa: E402

amd = pkgload.load()
rng = np.random.default_rng(1)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 114
G = rng.standard_normal((n, n + 8))
S = G @ G.T + n * np.eye(n)
b = rng.standard_normal(n)
ba = amd.LocalBA()
for i in range(6):
    x = ba.dense_solve(S, b)
print("residual", float(np.abs(S @ x - b).max()), flush=True)
