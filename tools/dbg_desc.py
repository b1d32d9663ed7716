"""Debug aid: descriptors of the extractor test's first frame, GPU vs oracle: per mismatching
keypoint its level, level coordinates, level size and Hamming distance.  Needs the GPU."""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import pkgload  # noqa: E402
import oracle_ref as O  # noqa: E402

amd = pkgload.load()
from orb_slam2_amd import synth  # noqa: E402

W, H, seed = 640, 480, 1592590337
img = synth.frame(synth.canvas(seed, W, H), W, H, 0)
ref = O.extract(O.params(1000), img, want_pyramid=True)
ex = amd.ORBextractor(1000, 1.2, 8, 20, 7, max_w=W, max_h=H)
kps, desc = ex(img)
lw, lh = ref["sizes"]
ham = np.unpackbits(desc ^ ref["desc"], axis=1).sum(1)
bad = np.nonzero(ham)[0]
print("keypoints", len(kps), "mismatching", len(bad))
for k in bad[:30]:
    l = int(kps["octave"][k])
    s = float(np.float32(1.2) ** l) if l else 1.0
    x, y = float(kps["x"][k]) / s, float(kps["y"][k]) / s
    print(f"k {k} level {l} x {x:.1f} y {y:.1f} size {lw[l]}x{lh[l]} angle {kps['angle'][k]:.3f} hamming {ham[k]}")
