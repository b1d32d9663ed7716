"""Timeline of the local-BA solves in a rocprofv3 kernel trace (tools/lba_timing.py under
rocprofv3 --kernel-trace): the LM loop's kernels grouped into optimize() calls (separated by
host gaps > 100 us), per group the span and summed kernel time, then per kernel name the mean
duration and the mean idle time before it."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")
       .replace("orbamd::", "")) for r in rows]
groups, cur = [], [ks[0]]
for k in ks[1:]:
    if k[0] - cur[-1][1] > 100_000:
        groups.append(cur)
        cur = []
    cur.append(k)
groups.append(cur)
big = [g for g in groups if len(g) > 20]
print(f"{len(groups)} groups, {len(big)} LM loops")
for g in big[-4:]:
    span = (g[-1][1] - g[0][0]) / 1e3
    busy = sum(e - b for b, e, _ in g) / 1e3
    print(f"  LM loop: {len(g)} kernels, span {span:.1f} us, busy {busy:.1f} us, idle {span - busy:.1f} us")
# host time between the LM loops of the last two solves
if len(big) >= 4:
    a, b = big[-4], big[-3]
    print(f"  host gap between optimize() calls: {(b[0][0] - a[-1][1]) / 1e3:.1f} us")
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
for g in big[-4:]:
    for j, (b0, e0, name) in enumerate(g):
        dur[name].append((e0 - b0) / 1e3)
        if j:
            gap[name].append((b0 - g[j - 1][1]) / 1e3)
print(f"  {'kernel':32s} {'n':>5s} {'mean us':>8s} {'idle before':>11s}")
for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    gg = gap.get(name, [0])
    print(f"  {name[:32]:32s} {len(v):5d} {sum(v) / len(v):8.2f} {sum(gg) / max(len(gg), 1):11.2f}")
