# final build (depth-2 chains): select probes and the production merge timeline
set -o pipefail
mkdir -p gpurun_out/r04m
timeout -k 10 300 python tools/trace_run.py --opt sel_prof=1 > gpurun_out/r04_sel_prof_final.txt 2>&1 || exit 1
STEPS="timeline" bash tools/r04_measure.sh > gpurun_out/r04m/tl_step.log 2>&1 || exit 2
