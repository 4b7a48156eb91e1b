#!/bin/bash
# rocprofv3 kernel stats of the headline bench (2 timed steps); args: tag [extra bench args]
set -o pipefail
TAG=${1:-prof}; shift
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp -o run -- python3 bench.py --steps 2 --warmup 1 "$@" > $O/bench.json 2> $O/bench.log
rc=$?
f=$(find $O/rp -name '*kernel_stats.csv' | head -1)
cp "$f" $O/kernel_stats.csv 2>/dev/null
python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d}  {r["Name"][:110]}')
PY
cat $O/bench.json
exit $rc
