#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/configs
O=gpurun_out/configs
timeout -k 10 400 python bench_configs.py gbdt --trees 10 --steps 1 --warmup 0 --trace $O/gbdt_trace.json > $O/gbdt_t.json 2> $O/gbdt_t.log
rc=$?
grep -v amdgpu.ids $O/gbdt_t.log
exit $rc
