"""Per-kernel and per-dispatch summary of a rocprofv3 kernel trace (tools/prof_run.sh)."""
import collections
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_bench/bench_kernel_trace.csv"
rows = list(csv.DictReader(open(path)))
by = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbamd::", "")
    key = (name, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    by[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for key, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    print(f"{key[0][:34]:34s} grid={key[1]:>7}x{key[2]:>5}x{key[3]:>4} calls={len(v):4d} avg_us={sum(v)/len(v):9.2f}")
