#!/bin/bash
# BASELINE configs 2-5 on one MI355X (config 1 is CPU plumbing); JSON lines -> gpurun_out/configs/
set -o pipefail
mkdir -p gpurun_out/configs
O=gpurun_out/configs
timeout -k 10 300 python bench_configs.py lr --steps 5 --warmup 2 > $O/lr.json 2> $O/lr.log &&
timeout -k 10 400 python bench_configs.py infer --steps 3 --warmup 1 > $O/infer.json 2> $O/infer.log &&
timeout -k 10 500 python bench_configs.py gbdt --trees 10 --steps 1 --warmup 1 > $O/gbdt10.json 2> $O/gbdt10.log &&
timeout -k 10 600 python bench_configs.py cv --steps 1 --warmup 0 > $O/cv.json 2> $O/cv.log
rc=$?
cat $O/*.json
exit $rc
