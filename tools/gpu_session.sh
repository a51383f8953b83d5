set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 300 python3 tools/round_check.py --corpus c3 --corpus c4 --k 5 > $O/rc_untied.jsonl 2> $O/rc.err || { tail $O/rc.err; exit 1; }
cat $O/rc_untied.jsonl
timeout -k 10 200 python3 tools/round_check.py --corpus c4 --k 5 --opt round_untied=0 > $O/rc_tiedonly.jsonl 2>> $O/rc.err || { tail $O/rc.err; exit 2; }
cat $O/rc_tiedonly.jsonl
timeout -k 10 200 python3 tools/trace_run.py --opt sel_prof=1 > $O/sel_prof.txt 2>&1 || { tail $O/sel_prof.txt; exit 3; }
grep "sel_prof: untied\|ended by" $O/sel_prof.txt
