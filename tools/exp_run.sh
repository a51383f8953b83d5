set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_run.py --cfg "" --cfg "merge_timing=0" --cfg "list_grid=64" --cfg "list_grid=256" > gpurun_out/abA.jsonl 2> gpurun_out/abA.err || exit 1
ZBPE_LIB=$PWD/zig-bpe_amd/zbpe/ab/libzbpe_lb4.so timeout -k 10 200 python -u tools/ab_run.py --cfg "" --cfg "merge_timing=0" > gpurun_out/abB.jsonl 2> gpurun_out/abB.err || exit 2
STEPS=prof bash tools/gpu_check.sh > gpurun_out/prof_step.log 2>&1 || exit 3
