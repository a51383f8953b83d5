#!/bin/bash
# GPU box: new-path parity tests, A/B, late-scan microbenchmark, probes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "neighbour or arena or c1 or synth_goldens or random_corpora or encode" > gpurun_out/gt.log 2>&1 || { tail -40 gpurun_out/gt.log; exit 1; }
tail -2 gpurun_out/gt.log
timeout -k 10 200 python -u tools/ab_run.py --reps 2 --cfg "" --cfg "list_nb=0" > gpurun_out/ab_head.jsonl 2> gpurun_out/ab_head.err || exit 3
cat gpurun_out/ab_head.jsonl
timeout -k 10 150 python -u tools/late_scan_bench.py --vocab 8000 20000 31000 --grid 0 > gpurun_out/lsb.jsonl 2> gpurun_out/lsb.err || exit 4
cat gpurun_out/lsb.jsonl
timeout -k 10 150 python -u tools/trace_run.py --opt sel_prof=1 > gpurun_out/trace.txt 2>&1 || exit 5
grep prof gpurun_out/trace.txt
