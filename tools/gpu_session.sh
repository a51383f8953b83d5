# round-6 GPU session: the sharded words case (world 4, hand-over at merge 190) against the oracle's sum of stream
# lengths, then the full -m gpu suite and the bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=${O:-gpurun_out/r06j}; mkdir -p $O
timeout -k 10 120 python3 tools/dist_case.py --world 4 --case 0 2>> $O/dc.err | grep -v Gloo > $O/one.json || exit 1
cut -c1-300 $O/one.json
O=$O STEPS="test bench" bash tools/measure.sh || exit 2
