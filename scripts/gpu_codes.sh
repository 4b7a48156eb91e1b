#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py -m gpu -q -x > gpurun_out/codes_tests.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 400 python bench/hist_micro.py --rows 1e8 --reps 2 --variants "codes,L0 T20 full   w v4 fast,L4 T20 full   w v4 fast" > gpurun_out/codes_micro.log 2>&1 || { echo micro failed; exit 1; }
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --trace gpurun_out/trace_codes.json > gpurun_out/codes_bench.log 2>&1 || { echo bench failed; exit 1; }
echo ok
