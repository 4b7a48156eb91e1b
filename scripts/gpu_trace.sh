#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --trace gpurun_out/trace_1e8.json > gpurun_out/trace_bench.log 2>&1 || { echo bench failed; exit 1; }
echo ok
