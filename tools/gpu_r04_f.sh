# byte-pair histogram (epoch spills): exactness tests and rate; select_next phase probes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -k pair_hist_bytes --timeout 250 --timeout-method thread > gpurun_out/pytest_hist_bytes.log 2>&1 || exit 1
timeout -k 10 300 python tools/hist_bench.py --at 0 > gpurun_out/hist_bytes2.jsonl 2>&1 || exit 2
timeout -k 10 300 python tools/trace_run.py --opt sel_prof=1 > gpurun_out/r04_sel_prof.txt 2>&1 || exit 3
LIBS="kp0 kp1" ROUNDS=3 bash tools/ab_libs.sh > gpurun_out/r04_ab_kp.txt 2>&1 || exit 4
cp gpurun_out/ab_libs.jsonl gpurun_out/r04_ab_kp.jsonl
VARIANTS="new new_tie_trust=1" bash tools/timeline_ab.sh > gpurun_out/tl_trust.log 2>&1 || exit 5
