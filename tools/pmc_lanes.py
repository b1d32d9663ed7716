"""Active-lane summary of a rocprofv3 PMC pass (tools/pmc_run.sh lanes SQ_THREAD_CYCLES_VALU
SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE) -> JSON read by bench.py.

active_lane_frac = SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64): rocprof's own derived
VALUUtilization (counter_defs.yaml, gfx950) — the fraction of lanes active over the VALU
instructions a kernel issued (0: all idle, 1: no divergence, full wavefronts).
usage: python tools/pmc_lanes.py OUT.json gpurun_out/pmc_lanes width=640 height=480 nfeatures=1000 frames_per_launch=128"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_provenance import provenance  # noqa: E402
from pmc_traffic import per_kernel  # noqa: E402


def main():
    out, d = sys.argv[1], sys.argv[2]
    config = dict(a.split("=", 1) for a in sys.argv[3:] if "=" in a)
    t = per_kernel(d)
    res = {"source": "rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE "
                     "--kernel-trace -- python3 bench.py (tools/pmc_run.sh lanes)",
           "definition": "active_lane_frac = SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU * 64) (rocprof VALUUtilization)",
           "config": config, "provenance": provenance(), "kernels": {}}
    for k, c in sorted(t.items()):
        e = {kk: round(v, 1) for kk, v in c.items()}
        act = c.get("SQ_ACTIVE_INST_VALU", 0.0)
        if act > 0:
            e["active_lane_frac"] = round(c.get("SQ_THREAD_CYCLES_VALU", 0.0) / (act * 64), 4)
        res["kernels"][k] = e
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v.get("active_lane_frac") for k, v in res["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main()
