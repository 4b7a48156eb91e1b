#!/bin/bash
# v4 integer-atomic histogram: GPU numerics, microbenchmark, then the headline bench at 1e8.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x > gpurun_out/v4_tests.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 300 python bench/hist_micro.py --rows 1e7 > gpurun_out/v4_micro.log 2>&1 || { echo micro failed; exit 1; }
for m in masked full; do
  CDNAML_RF_HIST=$m timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/v4_1e8_$m.log 2>&1 || { echo bench $m failed; exit 1; }
done
echo ok
