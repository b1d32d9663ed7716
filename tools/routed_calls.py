"""bench.py's routed-call latency rows alone (bench_single_calls + bench_routed_calls), for a quick
GPU check: python tools/routed_calls.py [--no-cpu]"""
import json
import pathlib
import sys
import types

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402

amd = pkgload.load()
args = types.SimpleNamespace(no_cpu="--no-cpu" in sys.argv, lba_kf=20, lba_points=3000)
dev = torch.device("cuda", 0)
print(json.dumps(bench.bench_single_calls(args, amd, dev), indent=1), flush=True)
