"""Timeline of the pipelined PCIe leg from a rocprofv3 kernel + memory-copy trace: per batch the H2D
copy span and the extraction / matching / pack kernel spans, and how much of each copy overlaps
kernels.  usage: pcie_trace_summary.py DIR"""
import csv
import glob
import sys

d = sys.argv[1]
kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
mt = glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True)
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-28:]) for r in csv.DictReader(open(kt))]
cs = []
if mt:
    for r in csv.DictReader(open(mt[0])):
        cs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Kind", "copy")),
                   int(r.get("Size", r.get("Bytes", 0)) or 0)))
ks.sort()
cs.sort()
big = [c for c in cs if c[3] >= 1 << 24]   # the 64-frame uploads
print(f"{len(ks)} kernels, {len(cs)} copies, {len(big)} >= 16 MiB")
t0 = big[-12][0] if len(big) >= 12 else (ks[0][0] if ks else 0)
ev = sorted([(a, b, n) for a, b, n in ks if a >= t0] + [(a, b, f"COPY {k} {n >> 20} MiB") for a, b, k, n in cs if a >= t0])
for a, b, n in ev[:140]:
    print(f"{(a - t0) / 1e3:9.1f} {(b - t0) / 1e3:9.1f} {(b - a) / 1e3:8.1f}  {n}")
