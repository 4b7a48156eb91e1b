#!/bin/bash
# PMC counters of the codes-compaction kernels during the headline bench (1 warmup + 1 step)
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_compact
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-include-regex "compact|partition5" -d $O/a -o a --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 > $O/a.log 2>&1 || { echo pmc a failed; tail $O/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT FETCH_SIZE --kernel-include-regex "compact|partition5" -d $O/b -o b --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 > $O/b.log 2>&1 || { echo pmc b failed; tail $O/b.log; exit 1; }
echo ok
