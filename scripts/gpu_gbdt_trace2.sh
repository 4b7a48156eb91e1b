#!/bin/bash
# GBDT (BASELINE config 4 shape) traced: 20 rounds, depth 8, 256 bins, 1e8 x 100
set -o pipefail
O=gpurun_out/configs
mkdir -p $O
timeout -k 10 400 python bench_configs.py gbdt --trees 20 --steps 1 --warmup 1 --trace $O/gbdt_trace.json > $O/gbdt_t.json 2> $O/gbdt_t.log
rc=$?
grep -v amdgpu.ids $O/gbdt_t.log | tail -30
cat $O/gbdt_t.json
exit $rc
