#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
timeout -k 10 300 python bench/hist_micro.py --rows 1e7 > gpurun_out/hist_micro_1e7.log 2>&1 || exit 1
timeout -k 10 300 python bench/hist_micro.py --rows 1e8 --reps 2 > gpurun_out/hist_micro_1e8.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 -i $GRAFT_REPO_ROOT/scripts/pmc_hist.txt --kernel-include-regex "hist" -d $GRAFT_REPO_ROOT/gpurun_out/pmc -o hist --output-format csv -- python $GRAFT_REPO_ROOT/bench/hist_micro.py --rows 1e7 --reps 1 > $GRAFT_REPO_ROOT/gpurun_out/pmc.log 2>&1
echo pmc exit $?
