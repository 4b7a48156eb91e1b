set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/run
run() {  # name rows env...
  local name=$1 rows=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --rows $rows --steps 8 --warmup 2 > gpurun_out/run/ab_$name.json 2> gpurun_out/run/ab_$name.log || exit 1
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/run/ab_$name.json) $(grep -o 'digest=[0-9a-f]*' gpurun_out/run/ab_$name.log | tail -1)"
}
run r8_base 1.25e7 CDNAML_LANE10_CHUNK3=0
run r8_c3 1.25e7 CDNAML_LANE10_CHUNK3=1
run r8_c3_m1024 1.25e7 CDNAML_LANE10_CHUNK3=1 CDNAML_SEG_MIN_BLOCKS=1024
run r8_c3_m512 1.25e7 CDNAML_LANE10_CHUNK3=1 CDNAML_SEG_MIN_BLOCKS=512
run r1_base 1e8 CDNAML_LANE10_CHUNK3=0
run r1_c3 1e8 CDNAML_LANE10_CHUNK3=1
run r1_c3_m1024 1e8 CDNAML_LANE10_CHUNK3=1 CDNAML_SEG_MIN_BLOCKS=1024
