#!/bin/bash
# GBDT config 4 in segment mode: 10-tree trace, then the full 500-tree run
set -o pipefail
mkdir -p gpurun_out/seg
O=gpurun_out/seg
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "seg" > $O/test.log 2>&1 &&
timeout -k 10 400 python bench_configs.py gbdt --trees 10 --steps 1 --warmup 0 --trace $O/gbdt_trace.json > $O/gbdt.json 2> $O/gbdt.log &&
timeout -k 10 600 python bench_configs.py gbdt --trees 500 --steps 1 --warmup 0 > $O/gbdt500.json 2> $O/gbdt500.log
rc=$?
tail -2 $O/test.log; grep -v amdgpu.ids $O/gbdt.log | tail -12; cat $O/gbdt500.json
exit $rc
