#!/bin/bash
# A/B of where the forest's Poisson bootstrap draws run in the fit prologue (profiles/r4/prologue_ab.md):
#   main       series on the main stream, right behind the quantile kernel (default)
#   side       side stream, queued at the same point (beside the binning)
#   side512    side stream, grid bounded to 512 blocks
#   main0      main stream, unbounded grid (T x 1024 blocks)
# gpurun --timeout 900 -- bash scripts/prologue_ab.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out/ab
mkdir -p "$O"
for rows in 1e8 1.25e7; do
  for v in main side side512 main0; do
    case $v in
      main) env_="CDNAML_POISSON_STREAM=main" ;;
      side) env_="CDNAML_POISSON_STREAM=side" ;;
      side512) env_="CDNAML_POISSON_STREAM=side CDNAML_POISSON_BLOCKS=512" ;;
      main0) env_="CDNAML_POISSON_STREAM=main CDNAML_POISSON_BLOCKS=0" ;;
    esac
    env $env_ timeout -k 10 300 python bench.py --rows $rows --steps 8 --warmup 1 > "$O/${v}_$rows.json" 2> "$O/${v}_$rows.log" || exit $?
    echo "$rows $v $(grep -o 'step [0-9.]* ms' "$O/${v}_$rows.log") $(grep -o 'digest=[0-9a-f]*' "$O/${v}_$rows.log")"
  done
done
