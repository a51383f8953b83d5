# round-6 GPU session: the full -m gpu suite and the bench line (tools/measure.sh), then the C3/C4 goldens with
# rounds outside list streaks (option round_streak 0) against the default
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=${O:-gpurun_out/r06d}; mkdir -p $O
O=$O STEPS="test bench" bash tools/measure.sh || exit 1
timeout -k 10 200 python3 tools/round_check.py --corpus c3 --corpus c4 --k 5 --opt round_streak=0 > $O/rc_streak0.jsonl 2>> $O/rc.err || { tail $O/rc.err; exit 2; }
cat $O/rc_streak0.jsonl
