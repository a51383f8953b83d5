# merges per device-resident batch (merge_batch 32 / 64 / 128) with pair selects: interleaved A/B
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r04_ab_batch.jsonl
for r in 1 2 3; do
  timeout -k 10 300 python -u tools/ab_run.py --reps 2 --cfg merge_batch=32 --cfg merge_batch=64 --cfg merge_batch=128 >> gpurun_out/r04_ab_batch.jsonl 2> gpurun_out/ab_b.err || exit 1
done
