# kernel trace of 200 KF solves (eager launches, fork mode): do the side-stream trailing updates
# overlap the next panel?
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
ORB_LBA_NO_GRAPH=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/mwtr -o run -- python3 $R/tools/lba_timing.py corridor=1 n_local=200 n_points=100000 solves=2 > $R/gpurun_out/mwtr.log 2>&1
cd $R
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/mwtr/*kernel_trace.csv")[0]
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("orbamd::","").replace("void ",""), r["Queue_Id"], r["Stream_Id"]) for r in csv.DictReader(open(f))]
rows.sort()
mw = [r for r in rows if "k_ldlt_mw_panel" in r[2] or "k_ldlt_mw_trail" in r[2]]
print("mw kernels", len(mw), "queues", sorted({(r[2][:18], r[3], r[4]) for r in mw})[:8])
ov = 0
for i in range(1, len(mw)):
    if mw[i][0] < mw[i-1][1]: ov += 1
print("overlapping consecutive pairs", ov, "of", len(mw) - 1)
seq = mw[-40:]
t0 = seq[0][0]
for r in seq[:16]:
    print(f"{r[2][:28]:28s} q{r[3]} s{r[4]} start {(r[0]-t0)/1000:8.2f} end {(r[1]-t0)/1000:8.2f} dur {(r[1]-r[0])/1000:6.2f}")
PY
