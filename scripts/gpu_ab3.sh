#!/bin/bash
# headline bench under several env settings (args: env assignments); no tests
set -o pipefail
O=gpurun_out/ab3
mkdir -p $O
i=0
for e in "$@"; do
  timeout -k 10 200 env $e python bench.py --steps 4 --warmup 1 > $O/r$i.json 2> $O/r$i.log || exit 1
  echo "$e: $(grep -o '"ms_per_step": [0-9.]*' $O/r$i.json)"
  i=$((i+1))
done
