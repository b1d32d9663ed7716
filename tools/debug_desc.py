import sys, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import numpy as np
import pkgload
amd = pkgload.load()
from orb_slam2_amd import synth
import oracle_ref as O
W, H = 640, 480
img = synth.frame(synth.canvas(0x5EED0001, W, H), W, H, 0)
ex = amd.ORBextractor(1000, 1.2, 8, 20, 7, max_w=W, max_h=H)
kps, desc = ex(img)
ref = O.extract(O.params(1000), img, want_pyramid=True)
bl0 = ref["blurred"][:W * H].reshape(H, W)
pat = np.array([int(t) for t in (ROOT / "orb-slam2-_amd/csrc/orb_pattern.inc").read_text().split("\n", 1)[1].replace(",", " ").split()]).reshape(256, 4)
def npdesc(im, kp):
    s, c = O.sincosf(np.float32(kp["angle"]) * np.float32(np.pi / 180))
    a, b = np.float32(c), np.float32(s)
    x, y = int(kp["x"]), int(kp["y"])
    bits = []
    for (x0, y0, x1, y1) in pat:
        g = lambda px, py: int(im[y + int(np.rint(np.float32(px) * b + np.float32(py) * a)), x + int(np.rint(np.float32(px) * a - np.float32(py) * b))])
        bits.append(g(x0, y0) < g(x1, y1))
    return np.packbits(np.array(bits, np.uint8), bitorder="little")
hd = [int(np.unpackbits(desc[i] ^ ref["desc"][i]).sum()) for i in range(min(20, len(desc)))]
print("hamming gpu vs ref", hd)
for i in range(3):
    print("gpu ", desc[i][:12])
    print("ref ", ref["desc"][i][:12])
    print("raw ", npdesc(img, kps[i])[:12])
    print("blur", npdesc(bl0, kps[i])[:12])
import ctypes as C
hip = C.CDLL("libamdhip64.so")
def dl(blurred, level):
    p = C.c_void_p(); w = C.c_int(); h = C.c_int(); pitch = C.c_size_t()
    rc = amd._abi.lib().orb_pyramid_level_device(ex._h, 0, level, blurred, C.byref(p), C.byref(w), C.byref(h), C.byref(pitch))
    out = np.zeros((h.value, pitch.value), np.uint8)
    hip.hipDeviceSynchronize()
    r = hip.hipMemcpy(out.ctypes.data_as(C.c_void_p), p, C.c_size_t(out.size), 2)
    return out[:, :w.value], r
g0, r = dl(1, 0)
print("memcpy rc", r, "gpu blur L0 vs oracle diff px:", np.count_nonzero(g0 != bl0))
idx = np.argwhere(g0 != bl0)[:10]
for (yy, xx) in idx:
    print(yy, xx, g0[yy, xx], bl0[yy, xx])
for i in range(3):
    print("from gpu blur", npdesc(g0, kps[i])[:12])
