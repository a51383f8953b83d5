#!/bin/bash
# GPU box: parity subset (incl. the >4 GiB sharded corpus), A/B vs the previous build (tools/ab_prep.sh; $CFGS: extra
# option sets of this build, space-separated), pipeline probes, kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
AB=zig-bpe_amd/zbpe/ab
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_dist.py -x -q --timeout 200 --timeout-method thread -k "tie or edge or neighbour or arena or c1 or synth_goldens or random_corpora or encode or sharded or bench" > gpurun_out/gt.log 2>&1 || { tail -40 gpurun_out/gt.log; exit 1; }
tail -2 gpurun_out/gt.log
ZBPE_LIB=$PWD/$AB/libzbpe_head.so timeout -k 10 150 python -u tools/ab_run.py --reps 2 --cfg "" > gpurun_out/ab_prev.jsonl 2> gpurun_out/ab_prev.err || exit 2
args=(--cfg ""); for c in $CFGS; do args+=(--cfg "$c"); done
timeout -k 10 250 python -u tools/ab_run.py --reps 2 "${args[@]}" > gpurun_out/ab_head.jsonl 2> gpurun_out/ab_head.err || exit 3
for v in $LIBS; do  # other builds of this tree (zig-bpe_amd/zbpe/ab/libzbpe_$v.so)
  ZBPE_LIB=$PWD/$AB/libzbpe_$v.so timeout -k 10 150 python -u tools/ab_run.py --reps 2 --cfg "" > gpurun_out/ab_$v.jsonl 2> gpurun_out/ab_$v.err || exit 4
  echo "== lib $v"; cat gpurun_out/ab_$v.jsonl
done
cat gpurun_out/ab_prev.jsonl gpurun_out/ab_head.jsonl
timeout -k 10 150 python -u tools/trace_run.py --opt sel_prof=1 > gpurun_out/trace.txt 2>&1 || exit 5
grep prof gpurun_out/trace.txt
rm -rf gpurun_out/prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 tools/ab_run.py --reps 1 --cfg "" > gpurun_out/prof_ab.jsonl 2> gpurun_out/prof.err || { tail gpurun_out/prof.err; exit 7; }
python3 tools/prof_summary.py gpurun_out/prof > gpurun_out/prof_summary.txt; head -24 gpurun_out/prof_summary.txt
find gpurun_out/prof -name "*kernel_trace.csv" -size +20M -delete
