#!/bin/bash
# Kernel-level profile of the headline bench at 1e8 rows (both histogram strategies).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for m in masked full; do
  CDNAML_RF_HIST=$m timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$m -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/prof_$m.log 2>&1 || { echo prof $m failed; exit 1; }
done
echo ok
