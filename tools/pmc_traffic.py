"""Per-launch HBM traffic per kernel from rocprofv3 PMC passes (tools/pmc_run.sh) -> JSON.

usage: python tools/pmc_traffic.py OUT.json fetch=gpurun_out/pmc_fetch write=gpurun_out/pmc_write \
           [raw=gpurun_out/pmc_raw] [--config KEY=VALUE ...]

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE
are collected in separate passes (TCC slots); FETCH_SIZE (KiB) counts 128-B requests at 64 B on
gfx950, so it is doubled; WRITE_SIZE (KiB) is taken as is. Infinity-Cache hits are counted by these
counters, so the figure is traffic below L2 (an upper bound on HBM bytes). An optional third pass
of the raw TCC_EA0_RDREQ / TCC_EA0_RDREQ_32B counters is summarised for cross-checking the units.
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_provenance import provenance  # noqa: E402


def per_kernel(d):
    files = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbamd::", "")
            name = name.split("<")[0].strip()
            acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[name].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in cs.items()} | {"dispatches": len(disp[k])}
            for k, cs in acc.items()}


def batches(table):
    """Extraction batches in the run: one k_fast_cell launch per batch (k_resize runs once per level)."""
    return table.get("k_fast_cell", {}).get("dispatches", 0)


def main():
    out = sys.argv[1]
    dirs, config = {}, {}
    for a in sys.argv[2:]:
        if a.startswith("--config"):
            continue
        k, v = a.split("=", 1)
        if k in ("fetch", "write", "raw"):
            dirs[k] = v
        else:
            config[k] = v
    fetch = per_kernel(dirs["fetch"])
    write = per_kernel(dirs["write"])
    raw = per_kernel(dirs["raw"]) if "raw" in dirs else {}
    kernels = {}
    nb = batches(fetch)
    for k in sorted(set(fetch) & set(write)):
        fk = fetch[k].get("FETCH_SIZE", 0.0)
        wk = write[k].get("WRITE_SIZE", 0.0)
        e = {"fetch_size_kib_raw": round(fk, 3), "write_size_kib": round(wk, 3),
             "read_bytes": round(2 * fk * 1024), "write_bytes": round(wk * 1024),
             "traffic_bytes_per_launch": round(2 * fk * 1024 + wk * 1024),
             "dispatches": fetch[k]["dispatches"]}
        if nb:
            # a bench "stage" may be several launches (k_resize: one per level); per-batch bytes
            # are what bench.py's stage timing divides by
            e["traffic_bytes_per_batch"] = round(e["traffic_bytes_per_launch"] * e["dispatches"] / nb)
        if k in raw:
            e["raw"] = {c: round(v, 1) for c, v in raw[k].items() if c != "dispatches"}
        kernels[k] = e
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) --kernel-trace",
           "correction": "read_bytes = 2 x FETCH_SIZE x 1024 (gfx950 128-B requests tallied at 64 B); "
                         "write_bytes = WRITE_SIZE x 1024",
           "config": config, "provenance": provenance(), "kernels": kernels}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for k, e in sorted(kernels.items(), key=lambda kv: -kv[1]["traffic_bytes_per_launch"]):
        print(f"{k[:30]:30s} read={e['read_bytes']/1e6:9.3f} MB write={e['write_bytes']/1e6:9.3f} MB "
              f"per launch ({e['dispatches']} launches)")


if __name__ == "__main__":
    main()
