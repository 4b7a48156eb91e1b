#!/bin/bash
# iterate: selected GPU tests, then kernel profile of the headline bench
set -o pipefail
O=gpurun_out/iter
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "${TESTS:-seg or codes or row_major}" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash scripts/gpu_prof.sh iterprof "$@"
