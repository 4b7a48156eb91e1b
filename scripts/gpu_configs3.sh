#!/bin/bash
# BASELINE configs 2-5 (1 GPU), JSON lines to gpurun_out/configs3/
set -o pipefail
O=gpurun_out/configs3
mkdir -p $O
timeout -k 10 200 python bench_configs.py lr --steps 5 --warmup 2 > $O/lr.json 2> $O/lr.log &&
timeout -k 10 300 python bench_configs.py cv --steps 1 --warmup 0 > $O/cv.json 2> $O/cv.log &&
timeout -k 10 300 python bench_configs.py infer --steps 3 --warmup 1 > $O/infer.json 2> $O/infer.log &&
timeout -k 10 500 python bench_configs.py gbdt --trees 500 --steps 1 --warmup 0 > $O/gbdt.json 2> $O/gbdt.log
rc=$?
cat $O/*.json
exit $rc
