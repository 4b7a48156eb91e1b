#!/bin/bash
# One parameterised GPU driver (replaces the round-1 one-off gpu_*.sh scripts).
#
#   gpurun --timeout 900 -- bash scripts/gpu.sh <step> [<step> ...]
#
# steps (run in order, chained: the first failure ends the call):
#   tests            pytest -m gpu (whole suite, one process)
#   tests:<expr>     pytest -m gpu -k <expr>
#   smoke            __graft_entry__.smoke()
#   bench            headline bench.py, 1e8 rows (5 timed steps)
#   bench8           per-rank shape of the 8-GPU point (1.25e7 rows)
#   prof             rocprofv3 --kernel-trace --stats of the headline step
#   prof8            same at 1.25e7 rows
#   pmc:<regex>      PMC pass (counters from scripts/pmc_hist.txt) over kernels matching <regex>
#   pmccfg:<regex>   same over one bench_configs.py config (CFG_ARGS: the config and its arguments)
#   configs          BASELINE configs 2-5 (bench_configs.py lr/cv/infer/gbdt)
#   cfg:<name>       one bench_configs.py config ('cfg:ooc --model rf': arguments after the name; outputs
#                    cfg_<name and arguments, non-alphanumerics as _>.json/.log)
#   profcfg:<name>   rocprofv3 --kernel-trace --stats of one bench_configs.py config (CFG_ARGS passed on)
#   py:<file>        python <file> (a scratch experiment)
# Extra environment for bench/prof steps: BENCH_ARGS="--steps 3 ..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out/run
mkdir -p "$O"
export TMPDIR=/tmp

kstats() {  # print the top of the first kernel_stats.csv under $1
    local f
    f=$(find "$1" -name "*kernel_stats.csv" | sort | sed -n 1p)
    [ -n "$f" ] && cut -c1-180 "$f" | sed -n 1,30p
}

run_step() {
    local s=$1
    case "$s" in
    tests)
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
            > "$O/tests.log" 2>&1; local rc=$?; tail -3 "$O/tests.log"; return $rc ;;
    tests:*)
        timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
            -k "${s#tests:}" > "$O/tests_k.log" 2>&1; local rc=$?; tail -15 "$O/tests_k.log"; return $rc ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
        timeout -k 10 400 python bench.py --steps 5 --warmup 1 ${BENCH_ARGS} > "$O/bench.json" 2> "$O/bench.log"
        local rc=$?; tail -3 "$O/bench.log"; cat "$O/bench.json"; return $rc ;;
    bench8)
        timeout -k 10 300 python bench.py --rows 1.25e7 --steps 5 --warmup 1 ${BENCH_ARGS} > "$O/bench8.json" 2> "$O/bench8.log"
        local rc=$?; tail -3 "$O/bench8.log"; cat "$O/bench8.json"; return $rc ;;
    prof|prof8)
        local rows=1e8; [ "$s" = prof8 ] && rows=1.25e7
        rm -rf "$O/$s"; mkdir -p "$O/$s"
        (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$s" -o p \
            -- python3 "$R/bench.py" --rows $rows --steps 2 --warmup 1 ${BENCH_ARGS} > "$O/$s/bench.log" 2>&1)
        local rc=$?; [ $rc -ne 0 ] && { tail -5 "$O/$s/bench.log"; return $rc; }
        kstats "$O/$s"
        python scripts/gaps.py "$(find "$O/$s" -name "*kernel_trace.csv" | sort | sed -n 1p)" > "$O/$s/gaps.txt"
        cat "$O/$s/gaps.txt" ;;
    profcfg:*)
        local c=${s#profcfg:}
        rm -rf "$O/profcfg"; mkdir -p "$O/profcfg"
        (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/profcfg" -o p \
            -- python3 "$R/bench_configs.py" $c ${CFG_ARGS} > "$O/profcfg/run.log" 2>&1)
        local rc=$?; [ $rc -ne 0 ] && { tail -5 "$O/profcfg/run.log"; return $rc; }
        kstats "$O/profcfg" ;;
    pmc:*)
        rm -rf "$O/pmc"; mkdir -p "$O/pmc"
        (cd /tmp && timeout -s KILL 300 rocprofv3 -i "$R/scripts/${PMC_FILE:-pmc_hist.txt}" --kernel-include-regex "${s#pmc:}" \
            --output-format csv -d "$O/pmc" -o p -- python3 "$R/bench.py" --steps 1 --warmup 0 ${BENCH_ARGS} \
            > "$O/pmc/run.log" 2>&1)
        local rc=$?; find "$O/pmc" -name "*counter_collection.csv"; return $rc ;;
    pmccfg:*)
        rm -rf "$O/pmccfg"; mkdir -p "$O/pmccfg"
        (cd /tmp && timeout -s KILL 300 rocprofv3 -i "$R/scripts/${PMC_FILE:-pmc_hist.txt}" --kernel-include-regex "${s#pmccfg:}" \
            --output-format csv -d "$O/pmccfg" -o p -- python3 "$R/bench_configs.py" ${CFG_ARGS} \
            > "$O/pmccfg/run.log" 2>&1)
        local rc=$?; find "$O/pmccfg" -name "*counter_collection.csv"; return $rc ;;
    configs)
        run_step cfg:lr && run_step cfg:cv && run_step cfg:infer && run_step cfg:gbdt ;;
    cfg:*)
        local c=${s#cfg:}; local nm; nm=$(echo "$c" | tr -c 'A-Za-z0-9_\n-' '_')
        timeout -k 10 600 python bench_configs.py $c ${CFG_ARGS} > "$O/cfg_$nm.json" 2> "$O/cfg_$nm.log"
        local rc=$?; tail -2 "$O/cfg_$nm.log"; cat "$O/cfg_$nm.json"; return $rc ;;
    py:*)
        timeout -k 10 600 python -u "${s#py:}" > "$O/py.log" 2>&1; local rc=$?; tail -30 "$O/py.log"; return $rc ;;
    *)
        echo "unknown step $s"; return 2 ;;
    esac
}

for s in "$@"; do
    echo "=== $s"
    run_step "$s" || { rc=$?; echo "step $s failed rc=$rc"; exit $rc; }
done
echo "all steps ok"
