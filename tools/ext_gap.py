"""What fills a stream's gap between its k_resolve_sfi and its next k_pyramid (rocprofv3 kernel trace of
the bench, tools/prof_run.sh): per stream its hardware queue, and per gap the kernels of ANY name that
ran on that stream inside it (torch copies, fills), the idle time, and which other streams' kernels
were running meanwhile.  usage: python tools/ext_gap.py gpurun_out/prof_bench/bench_kernel_trace.csv"""
import collections
import csv
import sys


def short(n):
    return n.split("(")[0].replace("void ", "").replace("orbamd::", "").split("<")[0].strip()[:40]


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Stream_Id"],
                     r["Queue_Id"]))
    rows.sort()
    n = len(rows)
    rows = rows[n // 5: n - n // 5]
    by_stream = collections.defaultdict(list)
    for r in rows:
        by_stream[r[3]].append(r)
    print("streams -> queues:", {s: sorted({r[4] for r in rs}) for s, rs in by_stream.items()})
    for s, rs in sorted(by_stream.items()):
        gaps = 0
        for i, r in enumerate(rs):
            if r[2] != "k_resolve_sfi":
                continue
            j = i + 1
            while j < len(rs) and rs[j][2] != "k_pyramid":
                j += 1
            if j >= len(rs):
                continue
            inside = rs[i + 1:j]
            t_a, t_b = r[1], rs[j][0]
            busy = sum(e - b for b, e, *_ in inside)
            others = collections.Counter()
            for b, e, name, st, q in rows:
                if st != s and b < t_b and e > t_a:
                    others[name] += (min(e, t_b) - max(b, t_a))
            print(f"stream {s}: gap {(t_b - t_a) / 1e3:8.1f} us, own kernels {[(x[2], round((x[1] - x[0]) / 1e3, 1)) for x in inside]}, "
                  f"own busy {busy / 1e3:.1f} us; others running (us): "
                  f"{ {k: round(v / 1e3, 1) for k, v in others.most_common(5)} }")
            gaps += 1
            if gaps >= 3:
                break


if __name__ == "__main__":
    main()
