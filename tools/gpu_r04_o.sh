# pair selects: third-smallest home by wave 0 or wave 4 (pair_m3w), refresh skip: parity, A/B, probes per variant
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_o.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -x -v -k "c4_full_sequence or c3_full_sequence or c3_every_tie" --timeout 500 --timeout-method thread > gpurun_out/pytest_large_o.log 2>&1 || exit 2
: > gpurun_out/r04_ab_pair5.jsonl
for r in 1 2 3; do
  timeout -k 10 250 python -u tools/ab_run.py --reps 2 --cfg pair_select=0 --cfg pair_select=1,pair_m3w=0 --cfg pair_select=1 >> gpurun_out/r04_ab_pair5.jsonl 2> gpurun_out/ab_pair.err || exit 4
done
timeout -k 10 300 python tools/trace_run.py --opt sel_prof=1 > gpurun_out/r04_sel_prof10.txt 2>&1 || exit 5
timeout -k 10 300 python tools/trace_run.py --opt sel_prof=1 --opt pair_m3w=0 > gpurun_out/r04_sel_prof10_w0.txt 2>&1 || exit 6
timeout -k 10 300 python tools/trace_run.py --opt sel_prof=1 --opt pair_select=0 > gpurun_out/r04_sel_prof10_off.txt 2>&1 || exit 7
