set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu.sh "tests:inference or graph_replayed" || exit $?
O=gpurun_out/run
timeout -k 10 600 python bench_configs.py infer --mode device --steps 3 --warmup 1 > $O/infer_dev.json 2> $O/infer_dev.log || { tail -5 $O/infer_dev.log; exit 1; }
tail -2 $O/infer_dev.log; cat $O/infer_dev.json
timeout -k 10 900 python bench_configs.py infer --mode host --steps 2 --warmup 1 > $O/infer_host.json 2> $O/infer_host.log || { tail -5 $O/infer_host.log; exit 1; }
tail -2 $O/infer_host.log; cat $O/infer_host.json
mkdir -p $O/infer_prof
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/infer_prof -o p -- python3 $GRAFT_REPO_ROOT/bench_configs.py infer --mode device --rows 2e8 --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/$O/infer_prof/log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/$O/infer_prof -name "*kernel_stats.csv" | xargs cut -c1-150 | head -8
