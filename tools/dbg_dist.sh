set -o pipefail
mkdir -p gpurun_out/r05d
O=gpurun_out/r05d/dist_dbg5.jsonl
for args in "--world 8 --case 13" "--world 8 --case 13 --opt debug_checks=1" "--world 8 --case 12 --opt replicate_late=0" "--world 8 --case 10"; do
  timeout -k 10 200 python3 tools/dist_case.py $args 2>> gpurun_out/r05d/dist_dbg5.err | grep -v Gloo >> $O || exit 1
done
grep -o '"world": [0-9]*, "case": [0-9]*, "options": {[^}]*}, "[a-z0-9]*": .\{0,240\}' $O
! grep -q '"error"\|"first_diff": [0-9]' $O
