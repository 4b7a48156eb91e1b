#!/bin/bash
# binize padded-table A/B: numerics (binize tests) under the flag, then the headline with and without it
set -o pipefail
O=gpurun_out/ab_binpad
mkdir -p $O
CDNAML_BINIZE_PAD=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "binize or quantile" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in pad base; do
  case $v in pad) E="CDNAML_BINIZE_PAD=1";; base) E="CDNAML_BINIZE_PAD=0";; esac
  env $E timeout -k 10 200 python bench.py --steps 4 --warmup 1 --trace $O/t_$v.json > $O/$v.json 2> $O/$v.log || exit 1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/$v.json) $(grep 'tree.binize' $O/$v.log)"
done
