#!/bin/bash
# GPU box: list-walk statistics, the late-scan microbenchmark, and the new bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 150 python -u tools/list_stats.py > gpurun_out/list_stats.txt 2>&1 || { tail gpurun_out/list_stats.txt; exit 1; }
timeout -k 10 150 python -u tools/late_scan_bench.py --vocab 8000 20000 31000 --grid 0 > gpurun_out/lsb.jsonl 2> gpurun_out/lsb.err || { tail gpurun_out/lsb.err; exit 2; }
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 3; }
