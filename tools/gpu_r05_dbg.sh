# round-5 pass: rounds (skipping decremented members) against the full C3/C4 goldens, the round end reasons
# (C4, round_k 4), the production timeline with halt windows, then the multi-rank tests with poisoned device
# allocations (ZBPE_POISON=1: a read of unwritten memory fails the same way every run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=${O:-gpurun_out/r05e}; mkdir -p $O
timeout -k 10 300 python3 tools/round_check.py --corpus c3 --corpus c4 --k 4 --k 1 > $O/round_check.jsonl 2> $O/round_check.err || { tail $O/round_check.err; exit 1; }
cat $O/round_check.jsonl
timeout -k 10 300 python3 tools/trace_run.py --opt sel_prof=1 --opt round_k=4 > $O/sel_prof_touch.txt 2>&1 || exit 2
grep "ended by\|ending touches" $O/sel_prof_touch.txt
O=$O STEPS=timeline bash tools/measure.sh || exit 3
python3 -c "import json;d=json.load(open('$O/merge_timeline.json'));print(json.dumps(d['halt_windows'])[:1500]);print({k:v for k,v in d.items() if k.endswith('wall')})"
ZBPE_POISON=1 timeout -k 10 700 python -u -m pytest tests/test_dist.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_dist_poison.log 2>&1
rc=$?
tail -15 $O/pytest_dist_poison.log
exit $rc
