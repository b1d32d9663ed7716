"""rocprofv3 --stats kernel_stats.csv -> the short text summary kept under profiles/.
usage: python tools/stats_summary.py STATS.csv OUT.txt "header line" """
import csv
import re
import sys


def short(name):
    m = re.search(r"orbamd::(k_\w+)", name)
    if m:
        t = re.search(r"k_\w+<(\w+)>", name)
        return m.group(1) + (f"<{t.group(1)}>" if t else "")
    return name.split("(")[0][:40]


rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
with open(sys.argv[2], "w") as f:
    f.write(sys.argv[3] + "\n(MI355X, ROCm 7.2)\n\n")
    for r in rows:
        f.write(f"{short(r['Name']):40s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs']) / 1e3:9.2f} "
                f"min_us={float(r['MinNs']) / 1e3:9.2f} total_ms={float(r['TotalDurationNs']) / 1e6:8.3f} "
                f"pct={100 * float(r['TotalDurationNs']) / tot:6.2f}\n")
