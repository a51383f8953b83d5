# select_next phase probes (sel_prof) on the current build: argmax, decision, refresh workgroups
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/trace_run.py --opt sel_prof=1 > gpurun_out/r04_sel_prof.txt 2>&1 || exit 1
