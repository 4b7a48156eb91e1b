#!/bin/bash
# K16/K17 tests + relational config with and without the hash path + kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/run
bash scripts/gpu.sh "tests:hash or dict_encode or relational_on_hash" || exit $?
timeout -k 10 600 python bench_configs.py relational --steps 3 --warmup 1 > $O/rel.json 2> $O/rel.log || { tail -5 $O/rel.log; exit 1; }
grep bench_configs $O/rel.log
CDNAML_HASH_MIN_ROWS=1000000000000 timeout -k 10 600 python bench_configs.py relational --steps 3 --warmup 1 > $O/rel_sort.json 2> $O/rel_sort.log || { tail -5 $O/rel_sort.log; exit 1; }
grep bench_configs $O/rel_sort.log
mkdir -p $O/rel_prof
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/rel_prof -o p -- python3 $GRAFT_REPO_ROOT/bench_configs.py relational --steps 1 --warmup 0 > $GRAFT_REPO_ROOT/$O/rel_prof/log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/$O/rel_prof -name "*kernel_stats.csv" | xargs cut -c1-140 | head -14
