#!/bin/bash
# GPU box measurement pass: parity (all -m gpu tests), the bench line, a rocprofv3 kernel trace of the
# bench command with the per-form scan roofline, the two PMC traffic passes, the production merge
# timeline (with the halt table), in-kernel probes. Each step has its own time limit; the first failure
# ends the script. STEPS picks steps, O the output directory (default gpurun_out/r05m), OPT engine
# options for the timeline / probe steps (e.g. OPT="--opt round_k=4").
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=${O:-gpurun_out/r05m}; mkdir -p $O
STEPS=${STEPS:-"test bench prof pmc timeline"}
for s in $STEPS; do
  case $s in
    test) timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
          tail -2 $O/pytest_gpu.log ;;
    bench) timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
           cat $O/bench.json ;;
    prof) rm -rf $O/prof
          timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
              python3 bench.py --steps 1 --warmup 0 --no-cpu --no-extra --scan-log-out $O/prof_scanlog.json > $O/prof_bench.json 2> $O/prof.err || { tail $O/prof.err; exit 3; }
          python3 tools/prof_summary.py $O/prof > $O/prof_summary.txt
          python3 tools/scan_forms.py $O/prof $O/prof_scanlog.json > $O/scan_forms.json || exit 4
          cat $O/scan_forms.json
          find $O/prof -name "*kernel_trace.csv" -size +20M -delete ;;
    pmc) OUT=$O bash tools/pmc_pass.sh > $O/pmc_step.log 2>&1 || { tail $O/pmc_step.log; exit 5; } ;;
    timeline) rm -rf $O/tl
          timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- \
              python3 tools/merge_timeline.py --run $O/tl_log.json $OPT > $O/tl.out 2>&1 || { tail $O/tl.out; exit 6; }
          python3 tools/merge_timeline.py --analyse $O/tl $O/tl_log.json > $O/merge_timeline.json || exit 7
          find $O/tl -name "*kernel_trace.csv" -size +20M -delete ;;
    probes) timeout -k 10 300 python3 tools/trace_run.py --opt sel_prof=1 $OPT > $O/sel_prof.txt 2>&1 || { tail $O/sel_prof.txt; exit 8; } ;;
    dist) ZBPE_LONG=1 timeout -k 10 1500 python -u -m pytest tests/test_dist.py -m gpu -v -s --durations=20 --timeout 1100 --timeout-method thread > $O/pytest_dist.log 2>&1 || { tail -30 $O/pytest_dist.log; exit 9; }
          grep HANDOVER $O/pytest_dist.log; tail -3 $O/pytest_dist.log ;;
  esac
done
