#!/bin/bash
# Generic GPU A/B: optional test selection, then interleaved headline benches over CDNAML_TUNE settings, then a
# kernel-stats profile of the first setting.
#   gpurun -- bash scripts/gpu_ab.sh "<pytest -k expr or ->" "<TUNE_A>" "<TUNE_B>" ["<TUNE_C>" ...]
# (ROWS=<n> in the environment sets the bench rows, default 1e8)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
O=$R/gpurun_out/run; mkdir -p "$O"; export TMPDIR=/tmp
K=$1; shift; A=$1; ROWS=${ROWS:-1e8}
if [ "$K" != "-" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" \
      > "$O/tests_ab.log" 2>&1 || { tail -40 "$O/tests_ab.log"; exit 1; }
  tail -2 "$O/tests_ab.log"
fi
for rep in 1 2; do
  for t in "$@"; do
    tag=$(echo "$t" | tr -c 'A-Za-z0-9\n' '_')
    CDNAML_TUNE="$t" timeout -k 10 300 python bench.py --rows $ROWS --steps 5 --warmup 1 > "$O/ab_$tag.json" 2> "$O/ab_$tag.log" || { tail -5 "$O/ab_$tag.log"; exit 1; }
    echo "[$t] $(grep 'step ' $O/ab_$tag.log)"
  done
done
rm -rf "$O/prof"; mkdir -p "$O/prof"
(cd /tmp && CDNAML_TUNE="$A" timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o p -- python3 "$R/bench.py" --rows $ROWS --steps 2 --warmup 1 > "$O/prof/bench.log" 2>&1) || exit 1
f=$(find "$O/prof" -name "*kernel_stats.csv" | sort | sed -n 1p)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f"{float(r['TotalDurationNs'])/3e6:8.2f} ms/step x{int(r['Calls'])/3:5.1f}  {r['Name'][:100]}")
PY
python scripts/gaps.py "$(find "$O/prof" -name "*kernel_trace.csv" | sort | sed -n 1p)" > "$O/prof/gaps.txt" && head -14 "$O/prof/gaps.txt"
