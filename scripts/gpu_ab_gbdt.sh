#!/bin/bash
# A/B: GBDT config (50 rounds) under two env settings (arg1 = env assignment for B)
set -o pipefail
O=gpurun_out/abg
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "${TESTS:-seg or compact}" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench_configs.py gbdt --trees 50 --steps 1 --warmup 0 > $O/a.json 2> $O/a.log || { tail $O/a.log; exit 1; }
timeout -k 10 300 env $1 python bench_configs.py gbdt --trees 50 --steps 1 --warmup 0 > $O/b.json 2> $O/b.log || { tail $O/b.log; exit 1; }
echo "A: $(grep -o '"ms_per_step": [0-9.]*' $O/a.json)"; echo "B ($1): $(grep -o '"ms_per_step": [0-9.]*' $O/b.json)"
