#!/bin/bash
# partition7 LDS-tile vs register-ladder bin lookup: numerics under the flag, then headline + per-rank shape
set -o pipefail
O=gpurun_out/ab_ladder
mkdir -p $O
CDNAML_PARTITION7_LADDER=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "partition" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in ladder tile; do
  case $v in ladder) E="CDNAML_PARTITION7_LADDER=1";; tile) E="CDNAML_PARTITION7_LADDER=0";; esac
  env $E timeout -k 10 200 python bench.py --steps 4 --warmup 1 --trace $O/t_$v.json > $O/$v.json 2> $O/$v.log || exit 1
  env $E timeout -k 10 200 python bench.py --rows 1.25e7 --steps 5 --warmup 1 --trace $O/t8_$v.json > $O/${v}_8.json 2> $O/${v}_8.log || exit 1
  echo "$v $(grep -ho '"ms_per_step": [0-9.]*' $O/$v.json $O/${v}_8.json | tr '\n' ' ') $(grep -h 'tree.partition' $O/$v.log $O/${v}_8.log | awk '{print $3}' | tr '\n' ' ')"
done
