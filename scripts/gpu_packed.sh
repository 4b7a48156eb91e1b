#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/pk_tests.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 400 python bench/hist_micro.py --rows 1e8 --reps 2 --variants "v5 packed,L0 T20 full   w v4 rot,L4 T20 full   w v4 rot" > gpurun_out/pk_micro.log 2>&1 || { echo micro failed; exit 1; }
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --trace gpurun_out/trace_pk.json > gpurun_out/pk_bench.log 2>&1 || { echo bench failed; exit 1; }
CDNAML_RF_HIST=masked timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/pk_bench_masked.log 2>&1 || { echo bench2 failed; exit 1; }
echo ok
