# round-4 first GPU pass: launch/barrier latencies, the dense histogram A/B, the quick GPU suite, the sharded C4 test
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/launch_lat > gpurun_out/launch_lat.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/hist_bench.py --at 0 --at 20000 > gpurun_out/hist_dense.jsonl 2>&1 || exit 2
timeout -k 10 300 python tools/hist_bench.py --at 0 --opt dense_hist=0 > gpurun_out/hist_hash.jsonl 2>&1 || exit 3
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_quick.log 2>&1 || exit 4
timeout -k 10 1100 python -u -m pytest tests/test_dist.py -x -v -m gpu -k c4_world2 --timeout 1050 --timeout-method thread > gpurun_out/pytest_dist_c4.log 2>&1 || exit 5
