set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu.sh tests:infer_udf && \
bash scripts/gpu.sh "cfg:infer --mode host --api transform" && \
bash scripts/gpu.sh "cfg:infer --mode host --api spark_udf" && \
bash scripts/gpu.sh "cfg:infer --mode device --api transform" && \
bash scripts/gpu.sh "cfg:infer --mode device --api spark_udf" && \
bash scripts/gpu.sh "cfg:ooc --model rf --trees 20 --source host --rows 2e8 --steps 1 --warmup 1"
