#!/bin/bash
# GPU box: parity (all gpu tests), A/B vs the round-1 build, late-scan microbenchmark, bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
AB=zig-bpe_amd/zbpe/ab
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gt.log 2>&1 || { tail -30 gpurun_out/gt.log; exit 1; }
tail -2 gpurun_out/gt.log
ZBPE_LIB=$PWD/$AB/libzbpe_r01.so timeout -k 10 150 python -u tools/ab_run.py --reps 2 --cfg "" > gpurun_out/ab_r01.jsonl 2> gpurun_out/ab_r01.err || exit 2
timeout -k 10 200 python -u tools/ab_run.py --reps 2 --cfg "" --cfg "list_nb=0" > gpurun_out/ab_head.jsonl 2> gpurun_out/ab_head.err || exit 3
cat gpurun_out/ab_r01.jsonl gpurun_out/ab_head.jsonl
timeout -k 10 150 python -u tools/late_scan_bench.py --vocab 8000 20000 31000 --grid 0 > gpurun_out/lsb.jsonl 2> gpurun_out/lsb.err || exit 4
timeout -k 10 150 python -u tools/trace_run.py --opt sel_prof=1 > gpurun_out/trace.txt 2>&1 || exit 5
