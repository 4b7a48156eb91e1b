#!/bin/bash
# GPU suite + GBDT (config 4 shape, 50 rounds) + XGBoost classifier smoke through K9
set -o pipefail
O=gpurun_out/check2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 400 python bench_configs.py gbdt --trees 50 --steps 1 --warmup 1 > $O/gbdt.json 2> $O/gbdt.log
rc=$?
tail -3 $O/pytest.log; grep -v amdgpu $O/gbdt.log | tail -3; cat $O/gbdt.json
exit $rc
