#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -m gpu -q -x > gpurun_out/rot_tests.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 400 python bench/hist_micro.py --rows 1e8 --reps 2 --variants "L0 T20 masked w v4,L0 T20 full   w v4,L4 T20 masked w v4,L4 T20 full   w v4" > gpurun_out/rot_micro.log 2>&1 || { echo micro failed; exit 1; }
for m in masked full; do
  CDNAML_HIST_MAP=4 CDNAML_RF_HIST=$m timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/rot_bench_$m.log 2>&1 || { echo bench failed; exit 1; }
done
echo ok
