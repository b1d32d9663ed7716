"""Does a pinned H2D copy overlap extraction kernels on another stream?  Times (a) 64-frame H2D
alone, (b) the 64-frame extraction alone, (c) both on two streams at once, (d) (c) with the copy
issued by hipMemcpyAsync through ctypes instead of torch — each over 10 repetitions."""
import ctypes as C
import sys
import time
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np
import torch
import pkgload

amd = pkgload.load()
from orb_slam2_amd import _abi, synth

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
W, H, B = 640, 480, 64
lib = _abi.lib()
cv = synth.canvas(7, W, H)
fr = np.stack([synth.frame(cv, W, H, t) for t in range(B)])
host = torch.from_numpy(fr).pin_memory()
d_copy = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
d_img = torch.from_numpy(fr).to(dev)
ex = amd.ORBextractor(1000, 1.2, 8, 20, 7, device=0, max_w=W, max_h=H, max_batch=B)
cap = C.c_int()
lib.orb_extractor_geometry(ex._h, W, H, None, None, None, C.byref(cap))
cap = cap.value
kps = torch.zeros((B, cap, 7), dtype=torch.int32, device=dev)
desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
cnt = torch.zeros(B, dtype=torch.int32, device=dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
hip = C.CDLL("libamdhip64.so")


def ext():
    _abi.check("x", lib.orb_extract_batch_device(ex._h, C.c_void_p(d_img.data_ptr()), H * W, B, W, H,
                                                  C.c_void_p(kps.data_ptr()), C.c_void_p(desc.data_ptr()), cap,
                                                  C.c_void_p(cnt.data_ptr()), C.c_void_p(s2.cuda_stream)))


def cp_torch():
    with torch.cuda.stream(s1):
        d_copy.copy_(host, non_blocking=True)


def cp_hip():
    r = hip.hipMemcpyAsync(C.c_void_p(d_copy.data_ptr()), C.c_void_p(host.data_ptr()), C.c_size_t(B * H * W), 1,
                           C.c_void_p(s1.cuda_stream))
    assert r == 0, r


def timed(fns, reps=10):
    for f in fns:
        f()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        for f in fns:
            f()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / reps * 1e3


print("h2d alone ms", round(timed([cp_torch]), 4))
print("h2d (hip) alone ms", round(timed([cp_hip]), 4))
print("extract alone ms", round(timed([ext]), 4))
print("both (torch copy) ms", round(timed([cp_torch, ext]), 4))
print("both (hip copy) ms", round(timed([cp_hip, ext]), 4))
