#!/bin/bash
# binize v6 (LUT) A/B: GPU tests of the binning kernel, then the headline with and without the LUT
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
O=$R/gpurun_out/run; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "binize or quantile or forest or heap" > "$O/tests_binize.log" 2>&1 || { tail -30 "$O/tests_binize.log"; exit 1; }
tail -2 "$O/tests_binize.log"
for v in 1 0 1 0; do
  CDNAML_TUNE=BINIZE_LUT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 1 > "$O/bench_lut$v.json" 2> "$O/bench_lut$v.log" || exit 1
  echo "LUT=$v $(grep 'step ' $O/bench_lut$v.log)"
done
rm -rf "$O/prof"; mkdir -p "$O/prof"
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o p -- python3 "$R/bench.py" --steps 2 --warmup 1 > "$O/prof/bench.log" 2>&1) || exit 1
f=$(find "$O/prof" -name "*kernel_stats.csv" | sort | sed -n 1p); grep -E "binize|root|lane10_kernel|partition7|predict_heap|scatter|count_w|poisson" "$f" | cut -c1-150
