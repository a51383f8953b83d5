# world-8 run-heavy case: which option removes the intermittent occurrence-count failure (14 runs each)
set -o pipefail
O=gpurun_out/r05l; mkdir -p $O
for opt in ""; do
  n=0
  for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
    timeout -k 10 120 python3 tools/dist_case.py --world 8 --case 10 $opt 2>> $O/rep.err | grep -v Gloo | cut -c1-500 > $O/one.json || exit 1
    grep -q '"error"' $O/one.json && n=$((n+1))
    cat $O/one.json >> $O/all.jsonl
  done
  echo "opt [$opt]: $n of 14 failed"
done
grep -h "error" $O/all.jsonl | grep -o "first 64.*" | head -5
