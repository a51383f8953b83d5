#!/bin/bash
# GPU box: where the late-merge kernels' time goes -- issue vs waiting, instruction fetch (two PMC passes over one
# production C4 train, zbpe_select_next / zbpe_replace / zbpe_scan_pairs_t) -> gpurun_out/pmc_ic_*.csv, summary
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_IFETCH SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
P3="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1)); rm -rf gpurun_out/pmc_ic$i
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "zbpe_select_next|zbpe_replace|zbpe_scan_pairs_t" --output-format csv \
      -d gpurun_out/pmc_ic$i -o run -- python3 tools/merge_timeline.py --run gpurun_out/pmc_ic$i.json > gpurun_out/pmc_ic$i.log 2>&1 \
      || { echo "pass $i failed"; tail -3 gpurun_out/pmc_ic$i.log; continue; }
  python3 tools/pmc_kernel_summary.py gpurun_out/pmc_ic$i > gpurun_out/pmc_ic$i.summary.json || true
  find gpurun_out/pmc_ic$i -name "*.csv" -size +20M -delete
done
cat gpurun_out/pmc_ic*.summary.json
