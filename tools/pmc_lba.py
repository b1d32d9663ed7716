"""Local-BA PMC summary (tools/gpu_lba_pmc.sh): per kernel, per launch, the f64 MFMA and VALU
counters of a rocprofv3 --pmc pass over tools/lba_timing.py -> JSON.

MfmaFlopsF64 = SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 (rocprofv3's derived-counter definition);
SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy cycles summed over SIMDs; GRBM_GUI_ACTIVE is the
kernel's GPU-active cycles.  The MFMA-busy fraction of the kernel's own SIMD (one workgroup
for k_ldlt_solve) is busy / GUI_ACTIVE; of the whole chip it is busy / (GUI_ACTIVE x 1024 SIMDs).
usage: python tools/pmc_lba.py OUT.json gpurun_out/pmc_lba_TAG [lba_timing.py args]"""
import json
import sys

sys.path.insert(0, __import__("pathlib").Path(__file__).resolve().parent.as_posix())
from pmc_traffic import per_kernel  # noqa: E402

out, d = sys.argv[1], sys.argv[2]
t = per_kernel(d)
res = {"source": "rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES "
                 "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 GRBM_GUI_ACTIVE --kernel-trace "
                 "-- python3 tools/lba_timing.py " + " ".join(sys.argv[3:]) + " (no args: config 4, 20 KF x 3000 points)",
       "env": {k: v for k, v in __import__("os").environ.items() if k.startswith("ORB_LBA_")},
       "kernels": {}}
for k, c in sorted(t.items()):
    e = {kk: round(v, 2) for kk, v in c.items()}
    mops = c.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0)
    e["mfma_flops_f64"] = int(mops * 512)
    gui = c.get("GRBM_GUI_ACTIVE", 0.0)
    busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    if gui > 0:
        e["mfma_busy_frac_chip"] = round(busy / (gui * 1024), 8)
    # VALU f64 flops: FMA counts 2 per lane-op, MUL/ADD 1; the counters are per wave instruction
    v = 2 * c.get("SQ_INSTS_VALU_FMA_F64", 0) + c.get("SQ_INSTS_VALU_MUL_F64", 0) + c.get("SQ_INSTS_VALU_ADD_F64", 0)
    e["valu_f64_flops"] = int(v * 64)
    res["kernels"][k] = e
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: {kk: v[kk] for kk in ("mfma_flops_f64", "valu_f64_flops", "dispatches") if kk in v}
                  for k, v in res["kernels"].items()}, indent=1))
