#!/bin/bash
# GPU box: tools/ab_run.py over the configurations in $AB (semicolon-separated), one line each -> gpurun_out/ab.jsonl
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
args=()
IFS=';' read -ra cfgs <<< "$AB"
for c in "${cfgs[@]}"; do args+=(--cfg "$c"); done
timeout -k 10 ${AB_TIMEOUT:-500} python -u tools/ab_run.py "${args[@]}" > gpurun_out/ab.jsonl 2> gpurun_out/ab.err
rc=$?
cat gpurun_out/ab.jsonl
[ $rc -ne 0 ] && tail -5 gpurun_out/ab.err
exit $rc
