#!/bin/bash
# kernel trace + PMC of the LinearRegression Gram (BASELINE config 2: 1e7 x 100 bf16)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/gram
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- python3 $R/bench_configs.py lr --steps 5 --warmup 2 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
grep bench_configs $O/kt.log
find $O/kt -name "*kernel_stats.csv" | xargs cut -c1-150 | head -5
timeout -s KILL 300 rocprofv3 -i $R/scripts/pmc_mfma.txt --kernel-include-regex "gram" --output-format csv -d $O/pmc -o p -- python3 $R/bench_configs.py lr --steps 1 --warmup 0 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
find $O/pmc -name "*counter_collection.csv"
