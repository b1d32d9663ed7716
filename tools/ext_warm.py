"""A few batched extractions of synthetic 640x480 frames (config 2) so the kernels run warm; with
the ORB_TIMING variant (tools/build_variant.py timing -DORB_TIMING, selected by ORB_SLAM2_AMD_LIB)
k_fast_cell and k_orient_desc print their in-kernel clock splits for a few cells / keypoints."""
import pathlib
import sys

import numpy as np
import torch

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import pkgload  # noqa: E402

amd = pkgload.load()
from orb_slam2_amd import synth  # noqa: E402

B, W, H, CAP = 64, 640, 480, 1200
cv = synth.canvas(1, W, H)
frames = torch.from_numpy(np.stack([synth.frame(cv, W, H, t) for t in range(B)])).cuda()
kps = torch.zeros((B, CAP * 7), dtype=torch.int32, device="cuda")
desc = torch.zeros((B, CAP, 32), dtype=torch.uint8, device="cuda")
cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
ex = amd.ORBextractor(1000, 1.2, 8, 20, 7, max_w=W, max_h=H, max_batch=B)
for it in range(3):
    print(f"-- batch {it}", flush=True)
    ex.extract_batch_device(frames, kps, desc, cnt)
    torch.cuda.synchronize()
print("keypoints frame 0:", int(cnt[0]), flush=True)
