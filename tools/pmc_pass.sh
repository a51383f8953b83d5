#!/bin/bash
# GPU box: HBM traffic of the scan kernel (two rocprofv3 PMC passes, one counter each) -> gpurun_out/pmc_traffic.json
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
export TMPDIR=/tmp
rm -rf $OUT/pmc_fetch $OUT/pmc_write
for c in FETCH_SIZE WRITE_SIZE; do
  d=$OUT/pmc_${c%%_SIZE}; d=${d,,}
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex zbpe_scan_pairs --output-format csv -d $d -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu --no-extra --scan-log-out $d.log.json > $d.json 2> $d.err || { echo "pmc $c failed rc=$?"; tail -5 $d.err; exit 1; }
done
python3 tools/pmc_traffic.py --fetch $OUT/pmc_fetch --fetch-log $OUT/pmc_fetch.log.json \
    --write $OUT/pmc_write --write-log $OUT/pmc_write.log.json > $OUT/pmc_traffic.json || exit 1
cat $OUT/pmc_traffic.json
find $OUT/pmc_fetch $OUT/pmc_write -name "*.csv" -size +30M -delete
