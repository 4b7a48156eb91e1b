#!/bin/bash
# Interleaved A/B of one bench_configs.py config under environment variants:
#   ab_cfg.sh "<config and args>" REPS "A=1" "B=2" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out/abcfg
mkdir -p "$O"
cfg=$1; reps=$2; shift 2
for r in $(seq 1 "$reps"); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    env $v timeout -k 10 600 python bench_configs.py $cfg > "$O/v${i}_r$r.json" 2> "$O/v${i}_r$r.log" || exit $?
    echo "[$v] rep $r: $(grep '^\[bench_configs\]' "$O/v${i}_r$r.log" | tail -1)"
  done
done
