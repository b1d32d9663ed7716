"""Debug aid: runs bench.py's extras legs, reading (and clearing) the HIP sticky error before and after
each leg, to name the leg that leaves a launch error behind."""
import ctypes as C
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.argv = ["bench.py", "--no-cpu"]
import torch  # noqa: E402
import bench  # noqa: E402

hip = C.CDLL("libamdhip64.so")
hip.hipGetErrorString.restype = C.c_char_p


def chk(tag):
    e = hip.hipGetLastError()
    print(f"{tag}: hipGetLastError = {e} {hip.hipGetErrorString(e).decode() if e else ''}", flush=True)


def wrap(name):
    f = getattr(bench, name)

    def g(*a, **k):
        chk(f"before {name}")
        r = f(*a, **k)
        torch.cuda.synchronize()
        chk(f"after {name}")
        return r
    setattr(bench, name, g)


for n in ("bench_stereo_kitti", "kitti_sfi_leg", "batch_sweep", "bench_pose", "bench_single_calls", "bench_bow",
          "bench_gba", "_extract_leg"):
    wrap(n)
args = bench.parse()
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
torch.cuda.set_stream(torch.cuda.Stream(dev))
amd = bench.pkgload.load()
chk("start")
try:
    bench.bench_extras(args, amd, dev)
finally:
    chk("end")
