"""Generates tests/golden/*.json: golden vectors of the CPU oracle on seeded
synthetic frames (inputs identified by SHA-256).  The reference ships no
fixtures of its own; these pin the oracle against regressions and
let GPU tests check the HIP path without re-running the oracle.
Run:  python tools/make_golden.py"""
import hashlib
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import numpy as np  # noqa: E402

import pkgload  # noqa: E402
import oracle_ref as O  # noqa: E402

CONFIGS = [("tum_640x480_1000", 640, 480, 1000, 0x5EED0001), ("mono_init_640x480_2000", 640, 480, 2000, 0x5EED0002),
           ("kitti_1241x376_2000", 1241, 376, 2000, 0x5EED0003), ("euroc_752x480_1200", 752, 480, 1200, 0x5EED0005)]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    pkgload.load()
    from orb_slam2_amd import synth
    out = {}
    for name, W, H, nf, seed in CONFIGS:
        cv = synth.canvas(seed, W, H)
        frames = [synth.frame(cv, W, H, t) for t in range(2)]
        p = O.params(nf)
        res = [O.extract(p, f) for f in frames]
        a, b = res
        fa, fb = O.FrameView(a["kps"], a["desc"], W, H), O.FrameView(b["kps"], b["desc"], W, H)
        prev = np.stack([a["kps"]["x"], a["kps"]["y"]], 1).astype(np.float32).reshape(-1)
        n, m12, prev2 = O.search_for_initialization(fa, fb, prev, nnratio=0.9, window=100)
        out[name] = {
            "W": W, "H": H, "nfeatures": nf, "seed": seed,
            "frames": [{
                "image_sha256": sha(f), "n": int(len(r["kps"])), "level_counts": r["level_counts"].tolist(),
                "pre_counts": r["pre_counts"].tolist(), "kps_sha256": sha(r["kps"]), "desc_sha256": sha(r["desc"]),
                "kps_head": [[float(k["x"]), float(k["y"]), float(k["size"]), float(k["angle"]), float(k["response"]),
                              int(k["octave"])] for k in r["kps"][:16]],
                "desc_head_hex": [bytes(d).hex() for d in r["desc"][:16]],
            } for f, r in zip(frames, res)],
            "sfi": {"nmatches": int(n), "matches12_sha256": sha(m12), "prev_sha256": sha(prev2)},
        }
        print(name, [fr["n"] for fr in out[name]["frames"]], n)
    (ROOT / "tests" / "golden" / "extract_match_golden.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
