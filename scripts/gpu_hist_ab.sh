#!/bin/bash
# A/B of histogram kernel versions / strategies on the RF benchmark.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "from cdnaml.ops import _lib; _lib.build(force=True)" > gpurun_out/ab_build.log 2>&1 || exit 1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu > gpurun_out/ab_tests.log 2>&1 || exit 1
for cfg in "1 masked 65536" "2 masked 65536" "2 masked 131072" "2 full 65536" "2 full 131072"; do
  set -- $cfg
  CDNAML_HIST_VERSION=$1 CDNAML_RF_HIST=$2 CDNAML_HIST_LDS=$3 timeout -k 10 300 python bench.py --rows 1e7 --steps 3 --warmup 1 > gpurun_out/ab_1e7_$1_$2_$3.log 2>&1 || exit 1
done
for cfg in "2 masked 65536" "2 full 65536"; do
  set -- $cfg
  CDNAML_HIST_VERSION=$1 CDNAML_RF_HIST=$2 CDNAML_HIST_LDS=$3 timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/ab_1e8_$1_$2_$3.log 2>&1 || exit 1
done
echo ok
