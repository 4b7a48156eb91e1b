#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/configs
O=gpurun_out/configs
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k gram > $O/gram_test.log 2>&1 &&
timeout -k 10 300 python bench_configs.py lr --steps 5 --warmup 2 > $O/lr.json 2> $O/lr.log
rc=$?
tail -3 $O/gram_test.log; cat $O/lr.json $O/lr.log | grep -v amdgpu.ids
exit $rc
