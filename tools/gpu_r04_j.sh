# lazy last-pair lookup (option lp_lazy): GPU parity suite, C3/C4 goldens, interleaved A/B, select probes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_j.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_large.py -x -q -k "c3_full_sequence or c4_full_sequence or c3_every_tie" --timeout 500 --timeout-method thread > gpurun_out/pytest_large_j.log 2>&1 || exit 2
: > gpurun_out/r04_ab_lp.jsonl
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/ab_run.py --reps 2 --cfg lp_lazy=0 --cfg lp_lazy=1 >> gpurun_out/r04_ab_lp.jsonl 2> gpurun_out/ab_lp.err || exit 3
done
timeout -k 10 300 python tools/trace_run.py --opt sel_prof=1 > gpurun_out/r04_sel_prof5.txt 2>&1 || exit 4
