#!/bin/bash
# One gpurun call's steps (edited per call): see tools/measure.sh for the steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06r; mkdir -p $O
LIBS="dppmax shflmax" ROUNDS=4 timeout -k 10 600 bash tools/ab_libs.sh > $O/ab_libs.txt 2>&1 || { tail $O/ab_libs.txt; exit 1; }
cat $O/ab_libs.txt; cp gpurun_out/ab_libs.jsonl $O/
O=$O STEPS="test bench" bash tools/measure.sh
