# late-merge grid sweep: per-merge timelines for the select's refresh grid and the list-scan grid
set -o pipefail
VARIANTS="new new_refresh_wgs=64 new_refresh_wgs=32 new_list_grid=256 new_list_grid=128" bash tools/timeline_ab.sh > gpurun_out/tl_sweep.log 2>&1
