# pair scans (a build with -DZBPE_PAIR_SCAN=1, zig-bpe_amd/zbpe/ab/libzbpe_ps.so): parity with it on, A/B, probes
set -o pipefail
mkdir -p gpurun_out
PS=$PWD/zig-bpe_amd/zbpe/ab/libzbpe_ps.so
ZBPE_LIB=$PS timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -x -v -k "pair" --timeout 500 --timeout-method thread > gpurun_out/pytest_pair_s.log 2>&1 || exit 1
: > gpurun_out/r04_ab_pscan.jsonl
for r in 1 2 3; do
  timeout -k 10 250 python -u tools/ab_run.py --reps 2 --cfg pair_select=1 >> gpurun_out/r04_ab_pscan.jsonl 2> gpurun_out/ab_ps.err || exit 2
  ZBPE_LIB=$PS timeout -k 10 250 python -u tools/ab_run.py --reps 2 --cfg pair_scan=0 --cfg pair_scan=1 >> gpurun_out/r04_ab_pscan.jsonl 2>> gpurun_out/ab_ps.err || exit 3
done
ZBPE_LIB=$PS timeout -k 10 300 python tools/trace_run.py --opt sel_prof=1 --opt pair_scan=1 > gpurun_out/r04_sel_prof14.txt 2>&1 || exit 4
