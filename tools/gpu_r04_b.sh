# dense histogram with rotated bins vs the hashed form; KP A/B of the C4 bench (kernarg preloading off/on)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/hist_bench.py --at 0 > gpurun_out/hist_dense2.jsonl 2>&1 || exit 2
timeout -k 10 300 python tools/hist_bench.py --at 0 --opt dense_hist=0 > gpurun_out/hist_hash2.jsonl 2>&1 || exit 3
