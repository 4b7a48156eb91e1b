set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/run
run() {  # name rows env...
  local name=$1 rows=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --rows $rows --steps 8 --warmup 2 > gpurun_out/run/ab_$name.json 2> gpurun_out/run/ab_$name.log || exit 1
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/run/ab_$name.json) $(grep -o 'digest=[0-9a-f]*' gpurun_out/run/ab_$name.log | tail -1)"
}
run r8_fill0 1.25e7 CDNAML_CODES_ROUND_FILL=0
run r8_fill1 1.25e7 CDNAML_CODES_ROUND_FILL=1
run r8_fill0b 1.25e7 CDNAML_CODES_ROUND_FILL=0
run r8_fill1b 1.25e7 CDNAML_CODES_ROUND_FILL=1
run r1_fill0 1e8 CDNAML_CODES_ROUND_FILL=0
run r1_fill1 1e8 CDNAML_CODES_ROUND_FILL=1
