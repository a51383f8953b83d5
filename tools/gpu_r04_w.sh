# argmax hot-list target (hot_target 1024 / 2048 / 4096) with pair selects: interleaved A/B
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r04_ab_hot.jsonl
for r in 1 2 3; do
  timeout -k 10 300 python -u tools/ab_run.py --reps 2 --cfg hot_target=1024 --cfg hot_target=2048 --cfg hot_target=4096 >> gpurun_out/r04_ab_hot.jsonl 2> gpurun_out/ab_h.err || exit 1
done
