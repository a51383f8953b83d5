#!/bin/bash
# GPU box: HBM traffic of the scan kernel (two rocprofv3 PMC passes, one counter each) -> gpurun_out/pmc_traffic.json
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
for c in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/pmc_${c%%_SIZE}; d=${d,,}
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex zbpe_scan_pairs --output-format csv -d $d -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu --scan-log-out $d.log.json > $d.json 2> $d.err || { echo "pmc $c failed rc=$?"; tail -5 $d.err; exit 1; }
done
python3 tools/pmc_traffic.py --fetch gpurun_out/pmc_fetch --fetch-log gpurun_out/pmc_fetch.log.json \
    --write gpurun_out/pmc_write --write-log gpurun_out/pmc_write.log.json > gpurun_out/pmc_traffic.json || exit 1
cat gpurun_out/pmc_traffic.json
find gpurun_out/pmc_fetch gpurun_out/pmc_write -name "*.csv" -size +30M -delete
