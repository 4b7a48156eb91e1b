#!/bin/bash
# segment-mode (single-tree) kernels: numerics, then GBDT config with trace
set -o pipefail
mkdir -p gpurun_out/seg
O=gpurun_out/seg
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "seg" > $O/test.log 2>&1 &&
timeout -k 10 400 python bench_configs.py gbdt --trees 10 --steps 1 --warmup 0 --trace $O/gbdt_trace.json > $O/gbdt.json 2> $O/gbdt.log
rc=$?
tail -5 $O/test.log; grep -v amdgpu.ids $O/gbdt.log | tail -14
exit $rc
