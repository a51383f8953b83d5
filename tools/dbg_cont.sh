# single-GPU trains of the run-heavy case under 8-process contention (96 runs), then the world-8 sharded case (14 runs)
set -o pipefail
O=gpurun_out/r05p2; mkdir -p $O
for i in 1 2; do
  timeout -k 10 250 python3 tools/contention_check.py --case 10 --procs 8 --reps 6 2>> $O/cont.err >> $O/cont.jsonl || exit 1
  tail -1 $O/cont.jsonl | cut -c1-400
done
n=0
for i in 1 2 3 4 5 6 7 8 9 10 11 12 13 14; do
  timeout -k 10 120 python3 tools/dist_case.py --world 8 --case 10 2>> $O/rep.err | grep -v Gloo | cut -c1-500 > $O/one.json || exit 1
  grep -q '"error"' $O/one.json && n=$((n+1))
  cat $O/one.json >> $O/all.jsonl
done
echo "world 8: $n of 14 failed"
