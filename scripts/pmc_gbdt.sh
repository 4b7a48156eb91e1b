# PMC pass over the GBDT config's lane4 histogram kernel (4 trees): bank conflicts vs LDS cycles
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out/run/pmc_gbdt
rm -rf "$O"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 300 rocprofv3 -i "$R/scripts/pmc_lane10.txt" --kernel-include-regex "seg_hist_lane4" \
    --output-format csv -d "$O" -o p -- python3 "$R/bench_configs.py" gbdt --trees 4 --steps 1 --warmup 0 \
    > "$O/run.log" 2>&1
rc=$?; find "$O" -name "*counter_collection.csv"; exit $rc
