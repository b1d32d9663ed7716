"""VALU / issue PMC summary of the extraction kernels (tools/gpu_valu_pmc.sh) -> JSON.

Per kernel, per launch: SQ_INSTS_VALU (wave-level VALU instructions), SQ_ACTIVE_INST_VALU,
SQ_BUSY_CYCLES, SQ_WAVE_CYCLES (quad-cycles, MI355X_MICROARCH.md "s_memtime tick vs SQ PMC units"),
SQ_WAVES, SQ_INSTS_LDS, SQ_INSTS_SALU, SQ_WAIT_INST_LDS, GRBM_GUI_ACTIVE (GPU-active cycles summed
over the 8 XCDs).  Derived:
  valu_lane_ops      = SQ_INSTS_VALU x 64 (every wave instruction occupies 64 lane slots);
  valu_peak          = 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 T lane-ops/s (a wave64 VALU
                       instruction issues over 2 cycles on a SIMD32);
  valu_frac(t)       = valu_lane_ops / (t x valu_peak), t = the launch's duration (the kernel-trace
                       average of the same pass and, in bench.py, the live HIP-event time);
  clock_ghz          = GRBM_GUI_ACTIVE / 8 / t (effective clock, DVFS included);
  valu_issue_util    = SQ_ACTIVE_INST_VALU x 4 / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): the fraction of
                       SIMD cycles that issued a VALU instruction while the kernel was active.
usage: python tools/pmc_valu.py OUT.json gpurun_out/pmc_valu [--config k=v ...]"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_provenance import provenance  # noqa: E402
from pmc_traffic import per_kernel  # noqa: E402

VALU_PEAK = 256 * 4 * 32 * 2.4e9


def kernel_durations(d):
    """Average kernel duration (ns) per kernel name from the pass's kernel trace."""
    files = glob.glob(os.path.join(d, "*kernel_trace.csv"))
    acc = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbamd::", "").split("<")[0].strip()
            t = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            s, n = acc.get(name, (0, 0))
            acc[name] = (s + t, n + 1)
    return {k: s / n for k, (s, n) in acc.items()}


def main():
    out, d = sys.argv[1], sys.argv[2]
    config = dict(a.split("=", 1) for a in sys.argv[3:] if "=" in a)
    t = per_kernel(d)
    dur = kernel_durations(d)
    res = {"source": "rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES "
                     "SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace",
           "valu_peak_lane_ops_per_s": VALU_PEAK, "config": config, "provenance": provenance(), "kernels": {}}
    for k, c in sorted(t.items()):
        e = {kk: round(v, 1) for kk, v in c.items()}
        ops = c.get("SQ_INSTS_VALU", 0.0) * 64
        e["valu_lane_ops"] = ops
        ns = dur.get(k)
        if ns:
            e["duration_ns_pmc_pass"] = round(ns, 1)
            e["valu_frac_pmc_pass"] = round(ops / (ns * 1e-9) / VALU_PEAK, 5)
            gui = c.get("GRBM_GUI_ACTIVE", 0.0)
            if gui:
                e["clock_ghz"] = round(gui / 8 / ns, 3)
                e["valu_issue_util"] = round(c.get("SQ_ACTIVE_INST_VALU", 0.0) * 4 / (gui / 8 * 1024), 4)
        res["kernels"][k] = e
    json.dump(res, open(out, "w"), indent=1)
    for k, e in res["kernels"].items():
        print(f"{k[:28]:28s} valu_ops={e['valu_lane_ops']/1e9:8.3f} G  frac={e.get('valu_frac_pmc_pass')}  "
              f"issue={e.get('valu_issue_util')}  clk={e.get('clock_ghz')}")


if __name__ == "__main__":
    main()
