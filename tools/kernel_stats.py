"""Format a rocprofv3 --stats kernel summary (bench_kernel_stats.csv) as the text table kept in profiles/."""
import csv
import sys

path, title = sys.argv[1], " ".join(sys.argv[2:])
print(title)
print("(MI355X, ROCm 7.2)\n")
for r in csv.DictReader(open(path)):
    name = r["Name"].split("(")[0].replace("orbamd::", "")
    print(f"{name[:40]:40s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs'])/1e3:9.2f} "
          f"total_ms={int(r['TotalDurationNs'])/1e6:8.3f} pct={float(r['Percentage']):6.2f}")
