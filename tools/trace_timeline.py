"""Print a window [N0, N1) of a rocprofv3 kernel + memory-copy trace as a timeline (start, end, duration
in us from the window start, stream, name).  usage: trace_timeline.py DIR N0 N1"""
import csv, glob, sys
d=sys.argv[1]; n0=int(sys.argv[2]); n1=int(sys.argv[3])
kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
mt = glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True)[0]
rows=[]
for r in csv.DictReader(open(kt)):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-22:], r.get("Stream_Id","?")))
for r in csv.DictReader(open(mt)):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY "+r["Direction"][12:], r["Stream_Id"]))
rows.sort()
t0=rows[n0][0]
for a,b,n,s in rows[n0:n1]:
    print(f"{(a-t0)/1e3:9.1f} {(b-t0)/1e3:9.1f} {(b-a)/1e3:8.1f} s{s} {n}")
