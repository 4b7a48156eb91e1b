#!/bin/bash
# Interleaved A/B of bench.py under environment variants: ab_env.sh ROWS REPS "A=1 B=2" "A=0" ...
# (each variant REPS times, round-robin, so clock / thermal drift spreads over all of them)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out/ab
mkdir -p "$O"
rows=$1; reps=$2; shift 2
for r in $(seq 1 "$reps"); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    env $v timeout -k 10 300 python bench.py --rows "$rows" --steps 8 --warmup 1 > "$O/v${i}_r$r.json" 2> "$O/v${i}_r$r.log" || exit $?
    echo "$rows [$v] rep $r: $(grep -o 'step [0-9.]* ms' "$O/v${i}_r$r.log") $(grep -o 'digest=[0-9a-f]*' "$O/v${i}_r$r.log")"
  done
done
