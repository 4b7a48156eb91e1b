set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/run
run() {  # name rows env...
  local name=$1 rows=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --rows $rows --steps 8 --warmup 2 > gpurun_out/run/ab_$name.json 2> gpurun_out/run/ab_$name.log || exit 1
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/run/ab_$name.json) $(grep -o 'digest=[0-9a-f]*' gpurun_out/run/ab_$name.log | tail -1)"
}
run r8_plain 1.25e7
run r8_overlap4 1.25e7 CDNAML_HIST_OVERLAP_FORCE=1
run r8_overlap2 1.25e7 CDNAML_HIST_OVERLAP_FORCE=1 CDNAML_HIST_OVERLAP=2
run r8_overlap4_mb1024 1.25e7 CDNAML_HIST_OVERLAP_FORCE=1 CDNAML_SEG_MIN_BLOCKS=1024
run r8_plain_b 1.25e7
