#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/pk5_tests.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 400 python bench/hist_micro.py --rows 1e8 --reps 2 --variants "128K" > gpurun_out/pk5_micro.log 2>&1 || { echo micro failed; exit 1; }
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --trace gpurun_out/trace_pk5.json > gpurun_out/pk5_bench.log 2>&1 || { echo bench failed; exit 1; }
echo ok
