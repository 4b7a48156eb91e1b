#!/bin/bash
# kernel-level profile of the headline step (1 warmup + 2 timed steps)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_headline
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_headline -o hl -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/prof_headline/bench.log 2>&1 || { echo prof failed; tail -5 $R/gpurun_out/prof_headline/bench.log; exit 1; }
find $R/gpurun_out/prof_headline -name "*kernel_stats.csv" | head -1 | xargs head -25
