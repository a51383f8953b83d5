# byte histogram (lean returning-add form) tests + rate; TLB-sized pointer chases
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -k pair_hist_bytes --timeout 250 --timeout-method thread > gpurun_out/pytest_hist_bytes.log 2>&1 || exit 1
timeout -k 10 300 python tools/hist_bench.py --at 0 > gpurun_out/hist_bytes3.jsonl 2>&1 || exit 2
timeout -k 10 200 ./tools/launch_lat > gpurun_out/launch_lat3.jsonl 2>&1 || exit 3
timeout -k 10 300 python tools/trace_run.py --opt sel_prof=1 > gpurun_out/r04_sel_prof2.txt 2>&1 || exit 4
