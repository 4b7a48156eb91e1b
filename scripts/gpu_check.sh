#!/bin/bash
# Full GPU check: test suite, smoke, headline bench (traced), and per-rank work of the 8-GPU strong-scaling case
set -o pipefail
O=gpurun_out/check
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --trace $O/trace.json > $O/bench.json 2> $O/bench.log &&
timeout -k 10 200 python bench.py --rows 1.25e7 --steps 5 --warmup 1 --trace $O/trace8.json > $O/bench_1p25e7.json 2> $O/bench_1p25e7.log
rc=$?
tail -3 $O/pytest.log; tail -2 $O/smoke.log; cat $O/bench.json $O/bench_1p25e7.json
exit $rc
