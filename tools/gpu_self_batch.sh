#!/bin/bash
# GPU box: self pairs inside batches -- the C3/C4 goldens, then one C4 train each with the option off and with a
# recount after every batch, then an interleaved A/B of the HEAD build (ab/libzbpe_head.so) against ab/libzbpe_sb.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=${O:-gpurun_out/sb}; mkdir -p $O
timeout -k 10 300 python3 tools/round_check.py --corpus c3 --corpus c4 --k 5 > $O/round_check.jsonl 2> $O/round_check.err || { tail $O/round_check.err; exit 1; }
cat $O/round_check.jsonl
AB_TIMEOUT=300 AB="self_batch=1;self_batch=0;batch_checks=1" bash tools/gpu_ab.sh > $O/ab_opts.jsonl 2>&1 || { tail $O/ab_opts.jsonl; exit 2; }
cat $O/ab_opts.jsonl
LIBS="head sb" ROUNDS=${ROUNDS:-3} bash tools/ab_libs.sh > $O/ab_libs.txt 2>&1 || { tail $O/ab_libs.txt; exit 3; }
cat $O/ab_libs.txt
