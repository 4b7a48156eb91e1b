#!/bin/bash
# multi-tree segment mode: kernel tests, then headline bench (traced) with and without it
set -o pipefail
O=gpurun_out/mseg
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "seg or codes or row_major" > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --trace $O/trace.json > $O/bench.json 2> $O/bench.log &&
timeout -k 10 200 python bench.py --rows 1.25e7 --steps 5 --warmup 1 --trace $O/trace8.json > $O/bench_1p25e7.json 2> $O/bench_1p25e7.log
rc=$?
tail -3 $O/pytest.log; grep -v amdgpu.ids $O/bench.log | tail -14; cat $O/bench.json $O/bench_1p25e7.json
exit $rc
