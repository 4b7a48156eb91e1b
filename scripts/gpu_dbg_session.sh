set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/run
CDNAML_HIP_DEBUG=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "seg10 or lane or e2e or forest or root" > gpurun_out/run/tests_dbg.log 2>&1; rc=$?; tail -2 gpurun_out/run/tests_dbg.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu.sh bench8 prof8
