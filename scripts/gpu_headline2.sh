#!/bin/bash
# kernel numerics touched this round + headline bench with trace
set -o pipefail
mkdir -p gpurun_out/hl2
O=gpurun_out/hl2
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -x > $O/test.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --trace $O/trace.json > $O/bench.json 2> $O/bench.log
rc=$?
tail -3 $O/test.log; grep -v amdgpu.ids $O/bench.log | tail -14; cat $O/bench.json
exit $rc
