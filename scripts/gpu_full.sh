#!/bin/bash
# full GPU suite + smoke + headline (1e8 and 1.25e7 per-rank) + GBDT 500 rounds
set -o pipefail
O=gpurun_out/full
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --trace $O/trace.json > $O/bench.json 2> $O/bench.log || exit 1
timeout -k 10 200 python bench.py --rows 1.25e7 --steps 5 --warmup 1 > $O/bench_1p25e7.json 2> $O/bench_1p25e7.log || exit 1
timeout -k 10 500 python bench_configs.py gbdt --trees 500 --steps 1 --warmup 0 > $O/gbdt.json 2> $O/gbdt.log || exit 1
grep -o '"ms_per_step": [0-9.]*' $O/bench.json $O/bench_1p25e7.json $O/gbdt.json
