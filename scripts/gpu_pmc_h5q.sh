#!/bin/bash
# PMC counters: lane-per-row packed kernel (hist5p) vs wave-compacted (hist5q) at L0 and L4
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 -i $R/scripts/pmc_hist.txt --kernel-include-regex "hist5" -d $R/gpurun_out/pmc_h5q -o h5 --output-format csv -- python3 $R/bench/hist_micro.py --rows 1e8 --reps 1 --variants "L0 T20 sub    codes pk8 128K,L0 T20 sub    codes pkq 128K,L4 T20 sub    codes pk8 128K,L4 T20 sub    codes pkq 128K" > $R/gpurun_out/pmc_h5q.log 2>&1 || { echo pmc failed; exit 1; }
echo ok
