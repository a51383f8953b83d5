#!/bin/bash
# GPU box, round-2 measurement pass: parity (all -m gpu tests), the bench line, a rocprofv3 kernel trace
# of the bench command with the per-form scan roofline, and the two PMC traffic passes. Each step has
# its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS=${STEPS:-"test bench prof pmc"}
for s in $STEPS; do
  case $s in
    test) timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
          tail -2 gpurun_out/pytest_gpu.log ;;
    bench) timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 2; }
           cat gpurun_out/bench.json ;;
    prof) rm -rf gpurun_out/prof
          timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
              python3 bench.py --steps 1 --warmup 0 --no-cpu --scan-log-out gpurun_out/prof_scanlog.json > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { tail gpurun_out/prof.err; exit 3; }
          python3 tools/prof_summary.py gpurun_out/prof > gpurun_out/prof_summary.txt
          python3 tools/scan_forms.py gpurun_out/prof gpurun_out/prof_scanlog.json > gpurun_out/scan_forms.json || exit 4
          cat gpurun_out/scan_forms.json
          find gpurun_out/prof -name "*kernel_trace.csv" -size +20M -delete ;;
    pmc) bash tools/pmc_pass.sh > gpurun_out/pmc_step.log 2>&1 || { tail gpurun_out/pmc_step.log; exit 5; } ;;
  esac
done
