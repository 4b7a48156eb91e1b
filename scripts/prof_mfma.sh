#!/bin/bash
# PMC + kernel trace of the MFMA level histogram alone (bench/mfma_micro.py --only mfma)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_mfma
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- python3 $R/bench/mfma_micro.py --rows 2e7 --nb 1 --reps 1 --only mfma > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
timeout -s KILL 300 rocprofv3 -i $R/scripts/pmc_mfma.txt --kernel-include-regex "hist_mfma_kernel" --output-format csv -d $O/pmc -o p -- python3 $R/bench/mfma_micro.py --rows 2e7 --nb 1 --reps 1 --only mfma > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
find $O -name "*counter_collection.csv" | head -3
find $O -name "*kernel_stats.csv" | xargs cut -c1-150 | head -6
