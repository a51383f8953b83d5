#!/bin/bash
# GPU box measurement pass: parity (all -m gpu tests), the bench line, a rocprofv3 kernel trace of the
# bench command with the per-form scan roofline, the two PMC traffic passes, the production merge
# timeline (with the halt table), in-kernel probes. Each step has its own time limit; the first failure
# ends the script. STEPS picks steps, O the output directory (default gpurun_out/r06m), OPT engine
# options for the timeline / probe steps (e.g. OPT="--opt round_k=4").
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=${O:-gpurun_out/r06m}; mkdir -p $O
STEPS=${STEPS:-"test bench prof pmc timeline"}
for s in $STEPS; do
  case $s in
    test) timeout -k 10 850 python -u -m pytest tests -m gpu -x -q --durations=25 --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
          tail -2 $O/pytest_gpu.log ;;
    bench) timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
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
    dist) timeout -k 10 1000 python -u -m pytest tests/test_dist.py -m gpu -v -s --durations=20 --timeout 600 --timeout-method thread > $O/pytest_dist.log 2>&1 || { tail -30 $O/pytest_dist.log; exit 9; }
          grep HANDOVER $O/pytest_dist.log; tail -3 $O/pytest_dist.log ;;
    # the full C3/C4 goldens for each round size K (K="1 5"), then the round end reasons (C4, round_k PK)
    rounds) KS=""; for k in ${K:-5}; do KS="$KS --k $k"; done
          timeout -k 10 400 python3 tools/round_check.py --corpus c3 --corpus c4 $KS > $O/round_check.jsonl 2> $O/round_check.err || { tail $O/round_check.err; exit 10; }
          cat $O/round_check.jsonl
          timeout -k 10 300 python3 tools/trace_run.py --opt sel_prof=1 --opt round_k=${PK:-5} > $O/sel_prof_rounds.txt 2>&1 || exit 11
          grep "ended by\|junction\|walks" $O/sel_prof_rounds.txt ;;
    # single-GPU run-heavy trains under 8-process contention (2 x 48), then the world-8 sharded case 14 times
    contention) for i in 1 2; do
            timeout -k 10 250 python3 tools/contention_check.py --case 10 --procs 8 --reps 6 2>> $O/cont.err >> $O/cont.jsonl || exit 12
            tail -1 $O/cont.jsonl | cut -c1-400
          done
          nf=0
          for i in $(seq 14); do
            timeout -k 10 120 python3 tools/dist_case.py --world 8 --case 10 2>> $O/rep.err | grep -v Gloo | cut -c1-500 > $O/one.json || exit 13
            grep -q '"error"' $O/one.json && nf=$((nf+1))
            cat $O/one.json >> $O/world8.jsonl
          done
          echo "world 8: $nf of 14 failed" ;;
    # production timeline with the kernels of every self-pair halt window below merge DUMP (default 2000)
    selfhalts) rm -rf $O/tl
          timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- \
              python3 tools/merge_timeline.py --run $O/tl_log.json $OPT > $O/tl.out 2>&1 || { tail $O/tl.out; exit 14; }
          python3 tools/merge_timeline.py --analyse $O/tl $O/tl_log.json --dump-self ${DUMP:-2000} > $O/merge_timeline.json 2> $O/self_halts.jsonl || exit 15
          rm -rf $O/tl ;;
  esac
done
