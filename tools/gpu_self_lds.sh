#!/bin/bash
# GPU box: the LDS-staged self-pair stream scan -- self-pair and sharded tests, the C3/C4 goldens, the halt
# timeline (zbpe_scan_self per halt), then an interleaved A/B against ab/libzbpe_head.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=${O:-gpurun_out/sl}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_dist.py -x -q -m gpu -k "self or sharded or encode" --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python3 tools/round_check.py --corpus c3 --corpus c4 --k 5 > $O/round_check.jsonl 2> $O/round_check.err || { tail $O/round_check.err; exit 2; }
cat $O/round_check.jsonl
O=$O/tl bash tools/gpu_self_halts.sh > $O/tl.txt 2>&1 || { tail $O/tl.txt; exit 3; }
python3 -c "
import json
for l in open('$O/tl/self_halts.jsonl'):
    d=json.loads(l); print(d['halt_merge'], {n: round(sum(k[1] for k in d['kernels'] if n in k[2]),1) for n in ('scan_self','self_tiles','self_carry')})
"
LIBS="head lds" ROUNDS=${ROUNDS:-3} bash tools/ab_libs.sh > $O/ab_libs.txt 2>&1 || { tail $O/ab_libs.txt; exit 4; }
cat $O/ab_libs.txt
