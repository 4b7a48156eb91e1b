#!/bin/bash
# Counters for the non-histogram kernels of the headline step.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 -i $R/scripts/pmc_hist.txt --kernel-include-regex "binize|partition5|predict" -d $R/gpurun_out/pmc_aux -o aux --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 > $R/gpurun_out/pmc_aux.log 2>&1 || { echo pmc failed; exit 1; }
echo ok
