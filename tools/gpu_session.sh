#!/bin/bash
# One gpurun call's steps (edited per call): see tools/measure.sh for the steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 60 tools/dpp_check > $O/dpp_check.txt 2>&1 || { cat $O/dpp_check.txt; exit 1; }
cat $O/dpp_check.txt
timeout -k 10 300 python3 tools/scan_bands.py --variants 0,7 > $O/scan_bands.jsonl 2> $O/scan_bands.err || { tail $O/scan_bands.err; exit 2; }
cat $O/scan_bands.jsonl
O=$O STEPS="test bench" bash tools/measure.sh
