#!/bin/bash
# One gpurun call's steps (edited per call): see tools/measure.sh for the steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 60 tools/dpp_check > $O/dpp_check.txt 2>&1 || { cat $O/dpp_check.txt; exit 1; }
cat $O/dpp_check.txt
O=$O STEPS="test bench prof timeline" bash tools/measure.sh
