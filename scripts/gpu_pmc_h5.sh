#!/bin/bash
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 -i $R/scripts/pmc_hist.txt --kernel-include-regex "hist5p" -d $R/gpurun_out/pmc_h5 -o h5 --output-format csv -- python3 $R/bench/hist_micro.py --rows 1e8 --reps 1 --variants "L0 T20 full   codes pk8 128K,L4 T20 full   codes pk8 128K" > $R/gpurun_out/pmc_h5.log 2>&1 || { echo pmc failed; exit 1; }
echo ok
