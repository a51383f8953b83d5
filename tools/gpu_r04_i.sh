# hcnt as a preloaded argument: parity (quick suite + the full C4 golden), select probes, A/B against the committed baseline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_i.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -x -v -k "c4_full_sequence or c4_prefix" --timeout 500 --timeout-method thread > gpurun_out/pytest_c4_full.log 2>&1 || exit 2
timeout -k 10 300 python tools/trace_run.py --opt sel_prof=1 > gpurun_out/r04_sel_prof4.txt 2>&1 || exit 3
LIBS="head hcnt" ROUNDS=3 bash tools/ab_libs.sh > gpurun_out/r04_ab_hcnt.txt 2>&1 || exit 4
cp gpurun_out/ab_libs.jsonl gpurun_out/r04_ab_hcnt.jsonl
bash tools/pmc_icache.sh > gpurun_out/r04_pmc_icache.txt 2>&1 || exit 5
bash tools/pmc_hist.sh > gpurun_out/r04_pmc_hist.txt 2>&1 || exit 6
