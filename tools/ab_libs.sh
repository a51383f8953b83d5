#!/bin/bash
# GPU box: interleaved A/B of library builds (zig-bpe_amd/zbpe/ab/libzbpe_<v>.so for v in $LIBS), $ROUNDS rounds of
# one tools/ab_run.py each (best of 3 C4 trains) -> gpurun_out/ab_libs.jsonl, then the median merges/s per build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out; : > gpurun_out/ab_libs.jsonl
for r in $(seq ${ROUNDS:-3}); do
  for v in $LIBS; do
    ZBPE_LIB=$PWD/zig-bpe_amd/zbpe/ab/libzbpe_$v.so timeout -k 10 120 python -u tools/ab_run.py --reps 2 --cfg "${CFG:-}" > gpurun_out/ab_one.jsonl 2> gpurun_out/ab_one.err || { tail -5 gpurun_out/ab_one.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab_one.jsonl').read().splitlines()[-1]);d['lib']='$v';d['round']=$r;print(json.dumps(d))" >> gpurun_out/ab_libs.jsonl
  done
done
python3 - <<'PY'
import json, statistics
rows = [json.loads(l) for l in open("gpurun_out/ab_libs.jsonl")]
for v in dict.fromkeys(r["lib"] for r in rows):
    xs = [r["merges_per_s"] for r in rows if r["lib"] == v]
    print(f"{v:8s} median {statistics.median(xs):9.1f} merges/s  all {[round(x) for x in xs]}  same_merges {all(r['same_merges'] for r in rows if r['lib'] == v)}")
PY
