"""Debug helper: compares the GPU extractor stage by stage with the oracle."""
import sys
import pathlib
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import numpy as np
import pkgload
amd = pkgload.load()
from orb_slam2_amd import synth
import oracle_ref as O

W, H = 640, 480
cv = synth.canvas(0x5EED0001, W, H)
img = synth.frame(cv, W, H, 0)
ex = amd.ORBextractor(1000, 1.2, 8, 20, 7, max_w=W, max_h=H)
kps, desc = ex(img)
ref = O.extract(O.params(1000), img, want_pyramid=True)
print("gpu N", len(kps), "ref N", len(ref["kps"]), "ref level counts", ref["level_counts"], "pre", ref["pre_counts"])
print("gpu per level", np.bincount(kps["octave"], minlength=8))
lw, lh = ref["sizes"]
off = 0
for lvl, a in enumerate(ex.mvImagePyramid):
    b = ref["pyramid"][off:off + lw[lvl] * lh[lvl]].reshape(lh[lvl], lw[lvl])
    off += lw[lvl] * lh[lvl]
    print("level", lvl, a.shape, "pyr diff px", np.count_nonzero(a != b))
n = min(len(kps), len(ref["kps"]))
for f in ("x", "y", "angle", "response", "octave"):
    print(f, "mismatch", np.count_nonzero(kps[f][:n] != ref["kps"][f][:n]))
print("desc mismatch rows", np.count_nonzero((desc[:n] != ref["desc"][:n]).any(1)))
print(kps[:5]); print(ref["kps"][:5])
