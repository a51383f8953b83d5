#!/bin/bash
# GPU box: production per-merge kernel timeline (tools/merge_timeline.py) of the A/B baseline library and of the working tree's
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VARIANTS:-head new}; do
  rm -rf gpurun_out/tl_$v
  # variant "head": the A/B baseline library; "new": the working tree's; "new_k=v": the working tree's with option k=v
  opt=()
  # "lib_<name>": zig-bpe_amd/zbpe/ab/libzbpe_<name>.so
  if [ $v = head ]; then export ZBPE_LIB=$PWD/zig-bpe_amd/zbpe/ab/libzbpe_head.so
  elif [ ${v#lib_} != $v ]; then export ZBPE_LIB=$PWD/zig-bpe_amd/zbpe/ab/libzbpe_${v#lib_}.so; else unset ZBPE_LIB; fi
  case $v in new_*) opt=(--opt "${v#new_}");; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$v -o run -- python3 tools/merge_timeline.py --run gpurun_out/tl_$v.json "${opt[@]}" > gpurun_out/tl_$v.log 2>&1 || { tail gpurun_out/tl_$v.log; exit 1; }
  python3 tools/merge_timeline.py --analyse gpurun_out/tl_$v gpurun_out/tl_$v.json > gpurun_out/tl_$v.out || exit 2
  find gpurun_out/tl_$v -name "*kernel_trace.csv" -delete
  echo "== $v"; cat gpurun_out/tl_$v.log; python3 -c "import json;d=json.load(open('gpurun_out/tl_$v.out'));k=list(d)[-1];print(k, json.dumps(d[k]))"
done
