#!/bin/bash
# GPU box: fused-scan parity tests, A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "fused or c1 or synth_goldens" > gpurun_out/gt.log 2>&1 || { tail -40 gpurun_out/gt.log; exit 1; }
tail -2 gpurun_out/gt.log
timeout -k 10 250 python -u tools/ab_run.py --reps 2 --cfg "" --cfg "fused_scan=1" > gpurun_out/ab_head.jsonl 2> gpurun_out/ab_head.err || { tail gpurun_out/ab_head.err; exit 3; }
cat gpurun_out/ab_head.jsonl
