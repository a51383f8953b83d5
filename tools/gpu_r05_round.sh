# multi-merge rounds: the full C3/C4 goldens for each round_k given (K="4 5"), then the round end reasons (C4)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=${O:-gpurun_out/r05f}; mkdir -p $O
KS=""; for k in ${K:-4}; do KS="$KS --k $k"; done
timeout -k 10 400 python3 tools/round_check.py --corpus c3 --corpus c4 $KS > $O/round_check.jsonl 2> $O/round_check.err || { tail $O/round_check.err; exit 1; }
cat $O/round_check.jsonl
timeout -k 10 300 python3 tools/trace_run.py --opt sel_prof=1 --opt round_k=${PK:-4} > $O/sel_prof.txt 2>&1 || exit 2
grep "ended by\|junction\|walks" $O/sel_prof.txt
