#!/bin/bash
# GPU tests (kernels + end-to-end estimators), headline bench, v4 histogram counters.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/r2_tests.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r2_bench.log 2>&1 || { echo bench failed; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 -i $R/scripts/pmc_hist.txt --kernel-include-regex "hist4" -d $R/gpurun_out/pmc_v4 -o hist --output-format csv -- python3 $R/bench/hist_micro.py --rows 1e8 --reps 1 --variants "L0 T20 masked w v4,L4 T20 masked w v4,L4 T20 full   w v4" > $R/gpurun_out/pmc_v4.log 2>&1 || { echo pmc failed; exit 1; }
echo ok
