#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/bp_tests.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --trace gpurun_out/trace_bp.json > gpurun_out/bp_bench.log 2>&1 || { echo bench failed; exit 1; }
echo ok
