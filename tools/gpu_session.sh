#!/bin/bash
# One gpurun call's steps (edited per call): see tools/measure.sh for the steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06t; mkdir -p $O
timeout -k 10 60 tools/dpp_check > $O/dpp_check.txt 2>&1 || { cat $O/dpp_check.txt; exit 1; }
cat $O/dpp_check.txt
LIBS="minK summ" ROUNDS=4 timeout -k 10 600 bash tools/ab_libs.sh > $O/ab_libs.txt 2>&1 || { tail $O/ab_libs.txt; exit 3; }
cat $O/ab_libs.txt; cp gpurun_out/ab_libs.jsonl $O/
O=$O STEPS="test" bash tools/measure.sh
