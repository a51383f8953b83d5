#!/bin/bash
# One gpurun call's steps (edited per call): see tools/measure.sh for the steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 400 python3 tools/ab_run.py --reps 2 --cfg "" --cfg sel_growth=8 --cfg sel_growth=4 --cfg sel_growth=0 --cfg sel_growth=0,hot_target=1024 > $O/ab_sel.jsonl 2> $O/ab_sel.err || { tail $O/ab_sel.err; exit 1; }
cat $O/ab_sel.jsonl
