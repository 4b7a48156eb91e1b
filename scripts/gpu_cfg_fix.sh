#!/bin/bash
# CV + GBDT configs after restricting partition7 to many-tree levels; partition7 min-T A/B on CV
set -o pipefail
O=gpurun_out/cfgfix
mkdir -p $O
timeout -k 10 300 python bench_configs.py cv --steps 1 --warmup 0 > $O/cv.json 2> $O/cv.log &&
CDNAML_PARTITION7_MIN_T=100 timeout -k 10 300 python bench_configs.py cv --steps 1 --warmup 0 > $O/cv_p5.json 2> $O/cv_p5.log &&
timeout -k 10 500 python bench_configs.py gbdt --trees 500 --steps 1 --warmup 0 > $O/gbdt.json 2> $O/gbdt.log
rc=$?
grep -h "CV\|GBDT" $O/*.log
exit $rc
