#!/bin/bash
# kernel trace of the per-rank work of the 8-GPU strong-scaling point (1.25e7 rows)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_1e8
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o p -- python3 $R/bench.py --steps 2 --warmup 1 > $O/bench.log 2>&1 || { echo prof failed; tail -5 $O/bench.log; exit 1; }
find $O -name "*kernel_stats.csv" | head -1 | xargs cut -c1-200 | head -40
