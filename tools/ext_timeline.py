"""Timeline of the bench's extraction steps from a rocprofv3 kernel trace (tools/prof_run.sh):
per stream, the busy fraction and the idle gaps between consecutive kernels; over all streams,
the fraction of wall time with at least one / two / three kernels running.  Answers whether a
step is bound by each stream's dependent chain (gaps, little overlap) or by the chip (overlap).
usage: python tools/ext_timeline.py gpurun_out/prof_bench/bench_kernel_trace.csv [first_kernel] [last_kernel]"""
import collections
import csv
import sys

EXT = ("k_pyramid", "k_fast_cell", "k_octree", "k_orient_desc", "k_grid_sfi", "k_cand_sfi", "k_resolve_sfi")


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbamd::", "").split("<")[0].strip()
        if name in EXT:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r["Stream_Id"], r["Queue_Id"]))
    rows.sort()
    if not rows:
        raise SystemExit("no extraction kernels in the trace")
    # the timed region: the last 60 % of the extraction dispatches (warm-up and the profiled pass excluded
    # crudely by taking the middle of the run)
    n = len(rows)
    rows = rows[n // 5: n - n // 5]
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    span = t1 - t0
    by_stream = collections.defaultdict(list)
    for r in rows:
        by_stream[r[3]].append(r)
    print(f"window {span / 1e3:.1f} us, {len(rows)} kernels, {len(by_stream)} streams")
    gaps_tot = collections.Counter()
    for s, rs in sorted(by_stream.items()):
        busy = sum(e - b for b, e, *_ in rs)
        gaps = collections.defaultdict(list)
        for a, b in zip(rs, rs[1:]):
            gaps[(a[2], b[2])].append(max(0, b[0] - a[1]) / 1e3)
        print(f"stream {s}: busy {busy / span:.3f} of the window, {len(rs)} kernels")
        for k, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:8]:
            print(f"   gap {k[0]:>14s} -> {k[1]:<14s} n={len(v):4d} avg_us={sum(v) / len(v):7.2f}")
            gaps_tot[k] += sum(v)
    ev = []
    for b, e, *_ in rows:
        ev += [(b, 1), (e, -1)]
    ev.sort()
    cover = collections.Counter()
    cur, last = 0, ev[0][0]
    for t, d in ev:
        cover[cur] += t - last
        cur += d
        last = t
    tot = sum(cover.values())
    print("concurrency (kernels running: fraction of the window):",
          {k: round(v / tot, 3) for k, v in sorted(cover.items())})
    dur = collections.defaultdict(list)
    for b, e, name, *_ in rows:
        dur[name].append((e - b) / 1e3)
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:16s} n={len(v):4d} avg_us={sum(v) / len(v):8.2f}")


if __name__ == "__main__":
    main()
