# round-6 GPU session: C3/C4 goldens (round_check), the kernel statistics of the bench command, then one PMC pass over
# the list build and select kernels of a C4 train (tools/pmc_rocpd.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=${O:-gpurun_out/r06g}; mkdir -p $O
timeout -k 10 200 python3 tools/round_check.py --corpus c3 --corpus c4 --k 5 > $O/rc.jsonl 2>> $O/rc.err || { tail $O/rc.err; exit 1; }
cat $O/rc.jsonl
O=$O STEPS="prof" bash tools/measure.sh > /dev/null || exit 2
head -25 $O/prof_summary.txt
rm -rf $O/pmc_build
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU \
    --kernel-include-regex "zbpe_list_scatter|zbpe_list_sort_scatter|zbpe_list_sort_hist|zbpe_pres_build|zbpe_select_next|zbpe_replace_round" \
    -d $O/pmc_build -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-extra > $O/pmc_build.log 2>&1 || { tail $O/pmc_build.log; exit 3; }
python3 tools/pmc_rocpd.py $O/pmc_build > $O/pmc_build.json; rm -rf $O/pmc_build $O/prof; cat $O/pmc_build.json
