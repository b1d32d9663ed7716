# one PMC pass: VALU instruction counts per kernel of the extraction step -> gpurun_out/pmc_vq
set -e
cd $GRAFT_REPO_ROOT
bash tools/pmc_run.sh vq SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES
python3 - <<'PY'
import csv, collections, glob
f = glob.glob('gpurun_out/pmc_vq/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].split('(')[0].split('::')[-1]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    if r['Counter_Name'] == 'SQ_INSTS_VALU': n[k] += 1
for k in sorted(acc, key=lambda k: -acc[k]['SQ_INSTS_VALU']):
    c = n[k] or 1
    print(f"{k:24s} launches={c:4d} VALU/launch={acc[k]['SQ_INSTS_VALU']/c:14.0f} LDS/launch={acc[k]['SQ_INSTS_LDS']/c:12.0f} SALU/launch={acc[k]['SQ_INSTS_SALU']/c:12.0f}")
PY
