#!/bin/bash
# One gpurun call's steps (edited per call): see tools/measure.sh for the steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06z; mkdir -p $O
for r in 1 2; do
timeout -k 10 400 python3 tools/ab_run.py --reps 2 --cfg "" --cfg refresh_wgs=128 --cfg refresh_wgs=64 --cfg refresh_wgs=32 >> $O/ab_refresh.jsonl 2>> $O/ab_refresh.err || { tail $O/ab_refresh.err; exit 1; }
done
cat $O/ab_refresh.jsonl | cut -c1-120
