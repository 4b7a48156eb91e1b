#!/bin/bash
# Round-1 closing measurements: headline (1e8) + per-rank 8-GPU shape, kernel stats of both, BASELINE configs 2-5
set -o pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --trace $O/trace.json > $O/bench.json 2> $O/bench.log &&
timeout -k 10 200 python bench.py --rows 1.25e7 --steps 5 --warmup 1 > $O/bench_1p25e7.json 2> $O/bench_1p25e7.log &&
bash scripts/gpu_prof_1e8b.sh > $O/prof1e8.txt 2>&1 &&
bash scripts/gpu_prof_8rank.sh > $O/prof8.txt 2>&1 &&
bash scripts/gpu_configs3.sh > $O/configs.txt 2>&1
rc=$?
cat $O/bench.json $O/bench_1p25e7.json; cat $O/configs.txt | tail -5
exit $rc
