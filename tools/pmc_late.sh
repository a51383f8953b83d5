#!/bin/bash
# GPU box: SQ counters of the late-phase merge kernels (one PMC pass; bench C4 train, 1 step) -> gpurun_out/late_pmc/
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/late_pmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_LDS \
    --kernel-include-regex "zbpe_replace|zbpe_select_next|zbpe_scan_pairs" --output-format csv -d gpurun_out/late_pmc -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/late_pmc.json 2> gpurun_out/late_pmc.err || { echo "pmc failed"; tail -5 gpurun_out/late_pmc.err; exit 1; }
python3 - <<'PY'
import csv, glob, collections
rows = collections.defaultdict(dict)
names = {}
for p in glob.glob("gpurun_out/late_pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        d = int(r["Dispatch_Id"])
        rows[d][r["Counter_Name"]] = rows[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[d] = r["Kernel_Name"].split("(")[0].split("<")[0].replace("zbpe::", "")
        rows[d]["grid"] = int(r["Grid_Size"]); rows[d]["wg"] = int(r["Workgroup_Size"])
ids = sorted(rows)[-6000:]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for d in ids:
    cnt[names[d]] += 1
    for k, v in rows[d].items(): agg[names[d]][k] += v
for n, a in agg.items():
    c = cnt[n]
    print(n, "dispatches", c, " ".join("%s=%.0f" % (k, v / c) for k, v in sorted(a.items())))
PY
find gpurun_out/late_pmc -name "*.csv" -size +30M -delete
