"""The pipelined PCIe-inclusive leg (bench._pcie_pipelined_leg, B = 64): the whole leg and its parts
(ORB_BENCH_PCIE_PART = copy: uploads only; compute: no uploads; nopack: no compaction into host
memory), and pipeline depths 3 / 4 (ORB_BENCH_PCIE_DEPTH), interleaved, in one process."""
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
    for part, depth in (("all", 3), ("all", 4), ("copy", 3), ("compute", 3), ("nopack", 3)):
        os.environ["ORB_BENCH_PCIE_DEPTH"] = str(depth)
        os.environ["ORB_BENCH_PCIE_PART"] = part
        r = bench._pcie_pipelined_leg(amd, dev, cv, 640, 480, 1000, 64)
        print("part", part, "depth", depth, "B 64", r["frames_per_s"], r["ms_per_step"], flush=True)
os.environ.pop("ORB_BENCH_PCIE_PART")
