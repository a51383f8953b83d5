# hot-list count mirror (Tables::hcnt): GPU parity suite, C3/C4 goldens, select probes, late-merge timeline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_h.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -x -q -k "c3_full_sequence or c4_prefix or c4_full_run or c3_every_tie" --timeout 500 --timeout-method thread > gpurun_out/pytest_large_h.log 2>&1 || exit 2
timeout -k 10 300 python tools/trace_run.py --opt sel_prof=1 > gpurun_out/r04_sel_prof3.txt 2>&1 || exit 3
VARIANTS="new" bash tools/timeline_ab.sh > gpurun_out/tl_hcnt.log 2>&1 || exit 4
