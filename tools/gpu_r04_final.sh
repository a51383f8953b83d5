# round-4 final pass on the default build: the new pair-option tests, the bench line, rocprof kernel trace +
# scan forms, PMC traffic, the merge timeline (tools/r04_measure.sh steps)
set -o pipefail
mkdir -p gpurun_out/r04m
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -x -v -k "pair or c4_full_sequence" --timeout 500 --timeout-method thread > gpurun_out/r04m/pytest_pair.log 2>&1 || exit 1
STEPS="bench prof pmc timeline" bash tools/r04_measure.sh > gpurun_out/r04m/measure.log 2>&1 || exit 2
