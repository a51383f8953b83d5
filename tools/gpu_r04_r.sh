# select kernel without calls (decide_body, block_max inlined: the NextArgs copy to scratch is gone): parity, A/B, probes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_large.py -x -v -k "c4_full_sequence or c3_full_sequence or c3_every_tie or c4_late_ties" --timeout 500 --timeout-method thread > gpurun_out/pytest_large_r.log 2>&1 || exit 2
timeout -k 10 300 python -u -m pytest tests/test_dist.py -x -v -m gpu -k sharded_c4 --timeout 250 --timeout-method thread > gpurun_out/pytest_dist_r.log 2>&1 || exit 3
: > gpurun_out/r04_ab_inline.jsonl
for r in 1 2 3; do
  timeout -k 10 250 python -u tools/ab_run.py --reps 2 --cfg pair_select=0 --cfg pair_chain=0 --cfg pair_chain=1 >> gpurun_out/r04_ab_inline.jsonl 2> gpurun_out/ab_pair.err || exit 4
done
timeout -k 10 300 python tools/trace_run.py --opt sel_prof=1 > gpurun_out/r04_sel_prof13.txt 2>&1 || exit 5
