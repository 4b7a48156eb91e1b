#!/bin/bash
# LR kernel profile + full 500-tree GBDT (BASELINE config 4)
set -o pipefail
mkdir -p gpurun_out/configs
O=$PWD/gpurun_out/configs
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_lr -o lr -- python3 $R/bench_configs.py lr --steps 5 --warmup 2 > $O/lr_prof.log 2>&1 &&
cd $R &&
timeout -k 10 600 python bench_configs.py gbdt --trees 500 --steps 1 --warmup 0 > $O/gbdt500.json 2> $O/gbdt500.log
rc=$?
find $O/prof_lr -name "*kernel_stats.csv" -exec head -20 {} \;
cat $O/gbdt500.json
exit $rc
