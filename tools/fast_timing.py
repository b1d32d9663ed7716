"""Per-phase clock64 stamps of the extraction kernels (ORB_TIMING variant): one 640x480 batch of
32 frames, extracted 3 times.  Build the variant first:
  python tools/build_variant.py timing -DORB_TIMING=1
and run with ORB_SLAM2_AMD_LIB=orb-slam2-_amd/lib/variant/timing/liborbslam2_amd.so."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT)]
import numpy as np  # noqa: E402
import pkgload  # noqa: E402

amd = pkgload.load()
from orb_slam2_amd import synth  # noqa: E402

W, H = 640, 480
cv = synth.canvas(0x5EED0001, W, H)
frames = np.stack([synth.frame(cv, W, H, t) for t in range(32)])
import torch  # noqa: E402
ex = amd.ORBextractor(1000, 1.2, 8, 20, 7, max_w=W, max_h=H, max_batch=32)
imgs = torch.from_numpy(frames).cuda()
cap = 4096
kps = torch.zeros((32, cap * 7), dtype=torch.int32, device="cuda")
desc = torch.zeros((32, cap, 32), dtype=torch.uint8, device="cuda")
cnt = torch.zeros(32, dtype=torch.int32, device="cuda")
for _ in range(3):
    ex.extract_batch_device(imgs, kps, desc, cnt)
    torch.cuda.synchronize()
print("done", cnt.cpu().numpy()[:4], flush=True)
