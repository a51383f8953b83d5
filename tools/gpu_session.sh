#!/bin/bash
# One gpurun call's steps (edited per call): see tools/measure.sh for the steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06w STEPS="test bench" bash tools/measure.sh
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06w/smoke.txt 2>&1 || { tail gpurun_out/r06w/smoke.txt; exit 5; }
tail -1 gpurun_out/r06w/smoke.txt
