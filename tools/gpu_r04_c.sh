# the byte-pair histogram: exactness tests, then its rate against the hashed form at C4 t = 0
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -k pair_hist_bytes --timeout 250 --timeout-method thread > gpurun_out/pytest_hist_bytes.log 2>&1 || exit 1
timeout -k 10 300 python tools/hist_bench.py --at 0 --at 20000 > gpurun_out/hist_bytes.jsonl 2>&1 || exit 2
timeout -k 10 300 python tools/hist_bench.py --at 0 --opt dense_hist=0 > gpurun_out/hist_hash3.jsonl 2>&1 || exit 3
timeout -k 10 120 ./tools/launch_lat > gpurun_out/launch_lat2.jsonl 2>&1 || exit 4
