#!/bin/bash
# GPU box: production timeline of a C4 train (tools/merge_timeline.py) with the kernels of every self-pair halt
# window below merge ${DUMP:-2000} -> $O/self_halts.jsonl
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=${O:-gpurun_out/sh}; mkdir -p $O; rm -rf $O/tl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- \
    python3 tools/merge_timeline.py --run $O/tl_log.json > $O/tl.out 2>&1 || { tail $O/tl.out; exit 6; }
python3 tools/merge_timeline.py --analyse $O/tl $O/tl_log.json --dump-self ${DUMP:-2000} > $O/merge_timeline.json 2> $O/self_halts.jsonl || exit 7
rm -rf $O/tl
python3 -c "import json;d=json.load(open('$O/merge_timeline.json'));print(json.dumps(d['halt_windows'])[:1500]);print({k:v for k,v in d.items() if k.endswith('halts')})"
