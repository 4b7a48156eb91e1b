#!/bin/bash
# what the driver runs at round end: GPU suite, smoke, default bench
set -o pipefail
O=gpurun_out/rehearsal
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.log
rc=$?
tail -1 $O/pytest.log; tail -1 $O/smoke.log; cat $O/bench.json
exit $rc
