#!/bin/bash
# GPU box, round-4 measurement pass: parity (all -m gpu tests), the bench line, a rocprofv3 kernel trace
# of the bench command with the per-form scan roofline, and the two PMC traffic passes. Each step has
# its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r04m; export TMPDIR=/tmp
STEPS=${STEPS:-"test bench prof pmc timeline"}
for s in $STEPS; do
  case $s in
    test) timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04m/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r04m/pytest_gpu.log; exit 1; }
          tail -2 gpurun_out/r04m/pytest_gpu.log ;;
    bench) timeout -k 10 400 python -u bench.py > gpurun_out/r04m/bench.json 2> gpurun_out/r04m/bench.err || { tail gpurun_out/r04m/bench.err; exit 2; }
           cat gpurun_out/r04m/bench.json ;;
    prof) rm -rf gpurun_out/r04m/prof
          timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04m/prof -o run -- \
              python3 bench.py --steps 1 --warmup 0 --no-cpu --no-extra --scan-log-out gpurun_out/r04m/prof_scanlog.json > gpurun_out/r04m/prof_bench.json 2> gpurun_out/r04m/prof.err || { tail gpurun_out/r04m/prof.err; exit 3; }
          python3 tools/prof_summary.py gpurun_out/r04m/prof > gpurun_out/r04m/prof_summary.txt
          python3 tools/scan_forms.py gpurun_out/r04m/prof gpurun_out/r04m/prof_scanlog.json > gpurun_out/r04m/scan_forms.json || exit 4
          cat gpurun_out/r04m/scan_forms.json
          find gpurun_out/r04m/prof -name "*kernel_trace.csv" -size +20M -delete ;;
    pmc) OUT=gpurun_out/r04m bash tools/pmc_pass.sh > gpurun_out/r04m/pmc_step.log 2>&1 || { tail gpurun_out/r04m/pmc_step.log; exit 5; } ;;
    timeline) rm -rf gpurun_out/r04m/tl
          timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04m/tl -o run -- \
              python3 tools/merge_timeline.py --run gpurun_out/r04m/tl_log.json > gpurun_out/r04m/tl.out 2>&1 || { tail gpurun_out/r04m/tl.out; exit 6; }
          python3 tools/merge_timeline.py --analyse gpurun_out/r04m/tl gpurun_out/r04m/tl_log.json > gpurun_out/r04m/merge_timeline.json || exit 7
          find gpurun_out/r04m/tl -name "*kernel_trace.csv" -size +20M -delete ;;
  esac
done
