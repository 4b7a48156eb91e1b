#!/bin/bash
# wave-compacted packed histogram: numerics, then per-level timing vs the lane-per-row kernel
set -o pipefail
mkdir -p gpurun_out/compact
O=gpurun_out/compact
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "hist_codes or partition" > $O/test.log 2>&1 &&
timeout -k 10 600 python bench/hist_micro.py --rows 1e8 --variants " sub " --reps 3 > $O/micro.txt 2>&1
rc=$?
tail -3 $O/test.log; cat $O/micro.txt | grep -v amdgpu.ids
exit $rc
