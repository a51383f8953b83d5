#!/bin/bash
# GPU box: parity tests (skipped with NOTEST=1), the scan rate by key density for $VARIANTS, and an
# A/B of train configurations $AB (tools/gpu_ab.sh). Each step has its own limit; stops at the first failure.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -3 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
fi
timeout -k 10 200 python -u tools/scan_density.py $((1 << 30)) ${VARIANTS:-0,2} || exit 1
AB="${AB:-;scan_auto=0}" bash tools/gpu_ab.sh
