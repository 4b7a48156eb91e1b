set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/run
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python bench_configs.py gbdt --trees 40 --steps 1 --warmup 1 > gpurun_out/run/gb_$name.json 2> gpurun_out/run/gb_$name.log || exit 1
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/run/gb_$name.json)"
}
run base
run prm CDNAML_PARTITION_RM=1
run base2
