#!/bin/bash
# PMC passes of the batched stream scan at three densities (one --pmc pass each, SQ counters only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06x; mkdir -p $O
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for pr in 1,0 104,97 46,32; do
  d=$O/pmc_${pr/,/_}
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex zbpe_scan_pairs --output-format csv -d $d -o run -- \
      python3 tools/scan_pmc.py --pair $pr --reps 10 --variant 7 > $d.json 2> $d.err || { echo "pmc $pr failed"; tail -5 $d.err; exit 1; }
  python3 tools/scan_pmc.py --summarise $d > $d.sum.json && cat $d.json $d.sum.json
  rm -rf $d
done
