"""Runs bench.py's global-BA leg alone (GPU box): python tools/gba_bench.py [--no-cpu]."""
import argparse
import json
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
import pkgload  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--no-cpu", action="store_true")
args = ap.parse_args()
amd = pkgload.load()
print(json.dumps(bench.bench_gba(args, amd, torch.device("cuda:0"))), flush=True)
