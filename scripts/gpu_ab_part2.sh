#!/bin/bash
# GPU suite, then partition7 vs partition8 on the headline and the 8-GPU per-rank shape
set -o pipefail
O=gpurun_out/ab_part2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in p8 p7; do
  case $v in p8) E="CDNAML_PARTITION8=1";; p7) E="CDNAML_PARTITION8=0";; esac
  env $E timeout -k 10 200 python bench.py --steps 4 --warmup 1 --trace $O/t_$v.json > $O/$v.json 2> $O/$v.log || exit 1
  env $E timeout -k 10 200 python bench.py --rows 1.25e7 --steps 5 --warmup 1 --trace $O/t8_$v.json > $O/${v}_8.json 2> $O/${v}_8.log || exit 1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/$v.json $O/${v}_8.json) $(grep 'tree.partition' $O/$v.log $O/${v}_8.log)"
done
