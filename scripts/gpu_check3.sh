#!/bin/bash
# full check: GPU suite, smoke, headline, per-rank 8-GPU shape, GBDT 50 rounds
set -o pipefail
O=gpurun_out/check3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > $O/bench.json 2> $O/bench.log &&
timeout -k 10 200 python bench.py --rows 1.25e7 --steps 5 --warmup 1 > $O/bench8.json 2> $O/bench8.log &&
timeout -k 10 400 python bench_configs.py gbdt --trees 50 --steps 1 --warmup 1 > $O/gbdt.json 2> $O/gbdt.log
rc=$?
tail -1 $O/pytest.log; tail -1 $O/smoke.log; grep -h "step " $O/bench.log $O/bench8.log; grep GBDT $O/gbdt.log
exit $rc
