#!/bin/bash
# Out-of-core RF fit streamed from pinned host chunks at 8e8 x 100 (320 GB of fp32 rows: more than HBM), 20 trees
# depth 5: the JSON line, then a rocprofv3 kernel + memory-copy trace of one fit and its H2D / kernel overlap.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
O=$R/gpurun_out/run; mkdir -p "$O"; export TMPDIR=/tmp
ROWS=${ROWS:-8e8}
ARGS="ooc --model rf --source host --rows $ROWS --trees 20 --steps 1 --warmup 1"
timeout -k 10 900 python bench_configs.py $ARGS > "$O/ooc8.json" 2> "$O/ooc8.log" || { tail -20 "$O/ooc8.log"; exit 1; }
tail -2 "$O/ooc8.log"; cat "$O/ooc8.json"
rm -rf "$O/ooc8prof"; mkdir -p "$O/ooc8prof"
(cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O/ooc8prof" -o p \
    -- python3 "$R/bench_configs.py" ooc --model rf --source host --rows $ROWS --trees 20 --steps 1 --warmup 0 \
    > "$O/ooc8prof/run.log" 2>&1) || { tail -20 "$O/ooc8prof/run.log"; exit 1; }
python scripts/copy_overlap.py "$O/ooc8prof" > "$O/ooc8prof/overlap.txt" && cat "$O/ooc8prof/overlap.txt"
