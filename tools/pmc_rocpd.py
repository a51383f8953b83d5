"""Per-kernel PMC summary from a rocprofv3 --pmc run's rocpd database (ROCm 7 writes SQLite by default):
  python3 tools/pmc_rocpd.py DIR [--skip-first]
Prints, per kernel name, the launches and the per-launch averages of every counter, plus the shares the SQ counters
give (wave-parked, issue-stalled, active; LDS bank conflicts per LDS-active cycle; VALU instructions per wave cycle)."""
import collections
import glob
import json
import os
import sqlite3
import sys


def main():
    d = sys.argv[1]
    skip = "--skip-first" in sys.argv
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        con = sqlite3.connect(db)
        for did, kn, cn, v in con.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
            short = kn.split("(")[0].replace("void ", "").replace("zbpe::", "")[:48]
            per[short][did][cn] = per[short][did].get(cn, 0.0) + v
    out = {}
    for k, disp in per.items():
        ids = sorted(disp)[1 if skip and len(disp) > 1 else 0:]
        tot = collections.defaultdict(float)
        for i in ids:
            for c, v in disp[i].items():
                tot[c] += v
        avg = {c: v / len(ids) for c, v in tot.items()}
        r = {"launches": len(ids), "per_launch": {c: round(v) for c, v in sorted(avg.items())}}
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU"):
                if c in avg:
                    r[c + "/SQ_WAVE_CYCLES"] = round(avg[c] / wc, 3)
        if avg.get("SQ_LDS_IDX_ACTIVE"):
            r["SQ_LDS_BANK_CONFLICT/SQ_LDS_IDX_ACTIVE"] = round(avg.get("SQ_LDS_BANK_CONFLICT", 0) / avg["SQ_LDS_IDX_ACTIVE"], 3)
        out[k] = r
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
