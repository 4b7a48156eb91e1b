#!/bin/bash
# PMC counters of binize2 / partition7 / codes_compact_w / predict_heap on the headline step (4 passes)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_r1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 -i $R/scripts/pmc_hist.txt --kernel-include-regex "binize2|partition7|codes_compact_w|predict_heap" -d $R/gpurun_out/pmc_r1 -o r1 --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 > $R/gpurun_out/pmc_r1/run.log 2>&1 || { echo pmc failed; tail -5 $R/gpurun_out/pmc_r1/run.log; exit 1; }
find $R/gpurun_out/pmc_r1 -name "*counter_collection.csv" | head
