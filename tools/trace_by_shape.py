"""Per (kernel, grid size) average durations from a rocprofv3 kernel_trace.csv."""
import collections
import csv
import re
import sys

g = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"orbamd::(k_\w+)", r["Kernel_Name"])
    name = m.group(1) if m else r["Kernel_Name"].split("(")[0][:30]
    grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    g[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (n, gr), v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
    print(f"{n:28s} grid={gr:9d} calls={len(v):4d} avg_us={sum(v) / len(v):9.2f} min_us={min(v):9.2f}")
