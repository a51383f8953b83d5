#!/bin/bash
# One GPU-box pass: parity tests, the bench line, option A/B, rocprof kernel stats. Each step has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-"test bench ab prof"}
rc=0
for s in $STEPS; do
  case $s in
    test) timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log ;;
    bench) timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; cat gpurun_out/bench.json ;;
    ab) timeout -k 10 400 python -u tools/ab_run.py $AB > gpurun_out/ab.jsonl 2> gpurun_out/ab.err; rc=$?; cat gpurun_out/ab.jsonl ;;
    enc) timeout -k 10 300 python -u tools/encode_bench.py > gpurun_out/encode.json 2> gpurun_out/encode.err; rc=$?; cat gpurun_out/encode.json ;;
    prof) rm -rf gpurun_out/prof; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_bench.json 2> gpurun_out/prof.err; rc=$?
          python3 tools/prof_summary.py gpurun_out/prof > gpurun_out/prof_summary.txt; head -20 gpurun_out/prof_summary.txt
          find gpurun_out/prof -name "*kernel_trace.csv" -size +20M -delete ;;
  esac
  if [ $rc -ne 0 ]; then echo "step $s failed rc=$rc"; tail -20 gpurun_out/*.err 2>/dev/null; exit $rc; fi
done
exit 0
