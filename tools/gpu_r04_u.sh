# pair-select chains of depth 3 (pair_chain=3): parity, A/B against the default depth 2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_large.py -x -v -k "pair or c4_full_sequence or c3_every_tie or c4_late_ties" --timeout 500 --timeout-method thread > gpurun_out/pytest_chain3.log 2>&1 || exit 1
: > gpurun_out/r04_ab_chain3.jsonl
for r in 1 2 3; do
  timeout -k 10 250 python -u tools/ab_run.py --reps 2 --cfg pair_chain=2 --cfg pair_chain=3 >> gpurun_out/r04_ab_chain3.jsonl 2> gpurun_out/ab_c3.err || exit 2
done
