#!/bin/bash
# One gpurun call's steps (edited per call): see tools/measure.sh for the steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06y; mkdir -p $O
for v in rec8 head rec8; do
  ZBPE_LIB=$PWD/zig-bpe_amd/zbpe/ab/libzbpe_$v.so timeout -k 10 300 python3 tools/scan_bands.py --variants 7 > $O/bands_$v.jsonl 2> $O/bands_$v.err || { tail $O/bands_$v.err; exit 2; }
  echo "== $v"; cat $O/bands_$v.jsonl
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_large.log 2>&1 || { tail -30 $O/pytest_large.log; exit 3; }
tail -2 $O/pytest_large.log
O=$O STEPS="bench" bash tools/measure.sh
