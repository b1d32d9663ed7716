"""N1 measurement: how often the build's creation-order tie-break
in DistributeOctTree's final phase (oracle_distribute_octree; csrc k_octree) differs from the
reference's (size, heap address) order under a real allocator.  oracle/n1_list_octree.cpp runs the
octree on a std::list of heap nodes in this process (glibc malloc) and sorts by pointer as
R/src/ORBextractor.cpp:736 does.  Per (frame, level): the same FAST keys (oracle_level_keys) go to
both; a level disagrees when the retained index sequences differ (order or content).  The same
std::list restatement run with creation-order ties must reproduce oracle_distribute_octree
exactly (checked on every level), so the differences are the tie-break alone.
This pins nothing: heap addresses depend on everything the process allocated before.
usage: python tools/n1_disagreement.py OUT.json [frames_per_config]"""
import ctypes as C
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import pkgload  # noqa: E402

pkgload.load()
from orb_slam2_amd import synth  # noqa: E402
import oracle_ref as O  # noqa: E402

n1 = C.CDLL(str(ROOT / "oracle" / "build" / "libn1_list_octree.so"))
n1.n1_list_octree.restype = C.c_int
P = O.P


def level_keys(p, img, w, h):
    cap = w * h // 4 + 64
    kx, ky, kr = (np.zeros(cap, np.float32) for _ in range(3))
    n = O.lib().oracle_level_keys(C.byref(p), P(np.ascontiguousarray(img)), w, h, P(kx), P(ky), P(kr), cap)
    return kx[:n], ky[:n], kr[:n]


def main():
    out = sys.argv[1]
    nfr = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    configs = [("640x480/1000 (config 2)", 640, 480, 1000, 0x5EED0002),
               ("1241x376/2000 (config 3)", 1241, 376, 2000, 0x5EED0003),
               ("752x480/1200 (config 5)", 752, 480, 1200, 0x5EED0005)]
    res = {"what": __doc__.split("\n")[0], "configs": {}}
    for name, W, H, NF, seed in configs:
        p = O.params(NF)
        t = O.tables(p)
        fpl = t["features_per_level"] if "features_per_level" in t else None
        cv = synth.canvas(seed, W, H)
        levels = dis = kp_total = kp_diff = same_set = 0
        per_level = np.zeros(8, np.int64)
        for f in range(nfr):
            ex = O.extract(p, synth.frame(cv, W, H, f), want_pyramid=True)
            lw, lh = ex["sizes"]
            offs = np.concatenate([[0], np.cumsum(lw.astype(np.int64) * lh)])
            for l in range(len(lw)):
                img = ex["pyramid"][offs[l]:offs[l + 1]].reshape(lh[l], lw[l])
                kx, ky, kr = level_keys(p, img, int(lw[l]), int(lh[l]))
                N = int(fpl[l]) if fpl is not None else int(ex["level_counts"][l])
                maxX, maxY = int(lw[l]) - 19 + 3, int(lh[l]) - 19 + 3
                a = O.distribute_octree(kx, ky, kr, 16, maxX, 16, maxY, N)
                b = np.zeros(len(kx) + 1, np.int32)
                nb = n1.n1_list_octree(P(kx), P(ky), P(kr), len(kx), 16, maxX, 16, maxY, N, 0, P(b))
                b = b[:nb]
                c = np.zeros(len(kx) + 1, np.int32)
                nc = n1.n1_list_octree(P(kx), P(ky), P(kr), len(kx), 16, maxX, 16, maxY, N, 1, P(c))
                if not np.array_equal(a, c[:nc]):
                    raise SystemExit(f"std::list restatement in creation order differs from the oracle ({name} f{f} l{l})")
                same_set += int(set(a.tolist()) == set(b.tolist()))
                levels += 1
                kp_total += len(a)
                if not np.array_equal(a, b):
                    dis += 1
                    per_level[l] += 1
                    kp_diff += len(set(a.tolist()) ^ set(b.tolist()))
        res["configs"][name] = {"frames": nfr, "levels": levels, "levels_disagreeing": dis,
                                "level_disagreement_rate": round(dis / levels, 4),
                                "levels_same_keypoint_set": same_set,
                                "disagreeing_levels_by_octave": per_level.tolist(),
                                "keypoints": kp_total, "keypoints_in_symmetric_difference": kp_diff,
                                "keypoint_disagreement_rate": round(kp_diff / max(kp_total, 1), 5)}
        print(name, res["configs"][name], flush=True)
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
