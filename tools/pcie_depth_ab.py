"""The pipelined PCIe-inclusive leg (bench._pcie_pipelined_leg, B = 8 and 64) at pipeline depths 3 / 4 / 5
(ORB_BENCH_PCIE_DEPTH: device frame buffers and host output sets in flight), interleaved, in one process."""
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402
import bench  # noqa: E402
import pkgload  # noqa: E402

amd = pkgload.load()
from orb_slam2_amd import synth  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
torch.cuda.set_stream(torch.cuda.Stream(dev))
cv = synth.canvas(0x5EED0002, 640, 480)
print("pinned copy GB/s", bench.measure_pinned_copy(dev), flush=True)
for rep in range(2):
    for depth in (3, 4, 5):
        os.environ["ORB_BENCH_PCIE_DEPTH"] = str(depth)
        for B in (8, 64):
            r = bench._pcie_pipelined_leg(amd, dev, cv, 640, 480, 1000, B)
            print("depth", depth, "B", B, r["frames_per_s"], r["ms_per_step"], flush=True)
