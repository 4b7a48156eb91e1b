#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "from cdnaml.ops import _lib; _lib.build(force=True)" > gpurun_out/v3_build.log 2>&1 || exit 1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu > gpurun_out/v3_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench/hist_micro.py --rows 1e7 > gpurun_out/v3_micro_1e7.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/v3_bench_1e8.log 2>&1 || exit 1
CDNAML_RF_HIST=full timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/v3_bench_1e8_full.log 2>&1 || exit 1
echo ok
