# pair selects, slack waves' loads issued together: parity (test_gpu + C4 full golden), A/B, probes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_l.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -x -v -k "c4_full_sequence or c3_full_sequence" --timeout 500 --timeout-method thread > gpurun_out/pytest_large_l.log 2>&1 || exit 2
: > gpurun_out/r04_ab_pair2.jsonl
for r in 1 2 3; do
  timeout -k 10 250 python -u tools/ab_run.py --reps 2 --cfg pair_select=0 --cfg pair_select=1 >> gpurun_out/r04_ab_pair2.jsonl 2> gpurun_out/ab_pair.err || exit 4
done
timeout -k 10 300 python tools/trace_run.py --opt sel_prof=1 > gpurun_out/r04_sel_prof7.txt 2>&1 || exit 5
timeout -k 10 300 python tools/trace_run.py --opt sel_prof=1 --opt pair_select=0 > gpurun_out/r04_sel_prof7_off.txt 2>&1 || exit 6
