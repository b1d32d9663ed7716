"""The pipelined PCIe-inclusive leg of bench.py (_pcie_pipelined_leg) in a fresh process, beside the serial leg and the pinned copy rates: whether its H2D / compute / D2H overlap."""
import sys
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch
import bench
import pkgload

amd = pkgload.load()
from orb_slam2_amd import synth

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
torch.cuda.set_stream(torch.cuda.Stream(dev))
cv = synth.canvas(0x5EED0002, 640, 480)
print("pinned copy GB/s", bench.measure_pinned_copy(dev))
m = amd.ORBmatcher(0.9, True, device=0)
print("serial B64", bench._pcie_leg(amd, dev, m, cv, 640, 480, 1000, 64)["frames_per_s"])
for rep in range(2):
    for B in (8, 64):
        r = bench._pcie_pipelined_leg(amd, dev, cv, 640, 480, 1000, B)
        print("pipelined B", B, r["frames_per_s"], r["ms_per_step"], r["d2h_bytes_per_step"])
print("serial B64", bench._pcie_leg(amd, dev, m, cv, 640, 480, 1000, 64)["frames_per_s"])
