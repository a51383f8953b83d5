#!/bin/bash
# GPU box: the full pair histogram at C4 t = 0 under rocprofv3 PMC passes, hashed form (dense_hist=0) vs the byte-bin
# form (dense_hist=1): LDS instructions / bank conflicts / VALU / waits, then FETCH_SIZE -> gpurun_out/pmc_hist_*.json
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out; export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"
for dense in 0 1; do
  for pass in 1 2; do
    if [ $pass = 1 ]; then P="$P1"; else P="FETCH_SIZE"; fi
    d=gpurun_out/pmc_hist_d${dense}_p$pass; rm -rf $d
    timeout -s KILL 200 rocprofv3 --pmc $P --kernel-include-regex "zbpe_pair_hist" --output-format csv -d $d -o run -- \
        python3 tools/hist_bench.py --at 0 --reps 3 --opt dense_hist=$dense > $d.log 2>&1 || { echo "pass d$dense p$pass failed"; tail -3 $d.log; exit 1; }
    python3 tools/pmc_kernel_summary.py $d 3 > $d.json || exit 2
  done
done
for f in gpurun_out/pmc_hist_d*_p*.json; do echo "== $f"; cat $f; done
