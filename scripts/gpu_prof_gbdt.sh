#!/bin/bash
# rocprofv3 kernel stats of 20 GBDT rounds (depth 8, 256 bins, 1e8 x 100)
O=$GRAFT_REPO_ROOT/gpurun_out/prof_gbdt
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp -o run -- python3 $GRAFT_REPO_ROOT/bench_configs.py gbdt --trees 20 --steps 1 --warmup 0 > $O/bench.json 2> $O/bench.log || { echo prof failed; tail $O/bench.log; exit 1; }
f=$(find $O/rp -name '*kernel_stats.csv' | head -1)
cp "$f" $O/kernel_stats.csv
python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:22]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d}  {r["Name"][:110]}')
PY
cat $O/bench.json
