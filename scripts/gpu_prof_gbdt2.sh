#!/bin/bash
# kernel trace of GBDT rounds (config 4 shape, 12 rounds)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_gbdt2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o g -- python3 $R/bench_configs.py gbdt --trees 12 --steps 1 --warmup 0 > $O/bench.log 2>&1 || { echo prof failed; tail -5 $O/bench.log; exit 1; }
find $O -name "*kernel_stats.csv" | head -1 | xargs cut -c1-150 | head -16
