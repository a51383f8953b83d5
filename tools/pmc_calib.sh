#!/bin/bash
# GPU box: FETCH_SIZE per scan launch on a known byte count (tools/pmc_calib.py) -> gpurun_out/calib*.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/calib
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex zbpe_scan_pairs --output-format csv -d gpurun_out/calib -o run -- \
    python3 tools/pmc_calib.py > gpurun_out/calib.json 2> gpurun_out/calib.err || { echo "calib failed"; tail -5 gpurun_out/calib.err; exit 1; }
cat gpurun_out/calib.json
python3 - <<'PY'
import csv, glob
for p in glob.glob("gpurun_out/calib/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        print(r["Dispatch_Id"], r["Kernel_Name"][:48], r["Counter_Name"], "%.4f GiB raw" % (float(r["Counter_Value"]) * 1024 / 2**30))
PY
