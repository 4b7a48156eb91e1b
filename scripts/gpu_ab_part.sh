#!/bin/bash
# A/B of the row-record partition variants on the headline (1e8 x 100, 20 trees, depth 5)
set -o pipefail
O=gpurun_out/ab_part
mkdir -p $O
for v in base p6 rm; do
  case $v in base) E="";; p6) E="CDNAML_PARTITION6=1";; rm) E="CDNAML_PARTITION_RM=1";; esac
  env $E timeout -k 10 200 python bench.py --steps 4 --warmup 1 --trace $O/t_$v.json > $O/$v.json 2> $O/$v.log || exit 1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/$v.json) $(grep 'tree.partition' $O/$v.log)"
done
