#!/bin/bash
# PMC counters for kernels matching $1 during a 1-step headline bench
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_$2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-include-regex "$1" -d $O/a -o a --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 > $O/a.log 2>&1 || { echo pmc a failed; tail $O/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE FETCH_SIZE --kernel-include-regex "$1" -d $O/b -o b --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 > $O/b.log 2>&1 || { echo pmc b failed; tail $O/b.log; exit 1; }
echo ok
