#!/bin/bash
# A/B of the wide-bin record-level block count for GBDT (40 trees, depth 8, 256 bins, 1e8 x 100)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/ab
for mb in 1024 512 256; do
  CDNAML_SEG_MIN_BLOCKS_WIDE=$mb timeout -k 10 300 python bench_configs.py gbdt --trees 40 --steps 1 --warmup 1 \
     > gpurun_out/ab/gbdt_mb$mb.json 2> gpurun_out/ab/gbdt_mb$mb.log || exit $?
  echo "mb=$mb $(grep 'ms/tree' gpurun_out/ab/gbdt_mb$mb.log)"
done
