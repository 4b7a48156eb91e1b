set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof1
timeout -k 10 300 python __graft_entry__.py > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --rows 1e7 --steps 3 --warmup 1 > gpurun_out/bench_1e7.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_1e8.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --rows 1e7 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1
echo done $?
