#!/bin/bash
# binize2 kernel time vs rows per tile (rocprofv3 kernel trace of a 1e8 x 100 x 40-bin binning)
O=$GRAFT_REPO_ROOT/gpurun_out/rpt
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for r in 64 32 16; do
  CDNAML_BINIZE_RPT=$r timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r$r -o run -- python3 -c "
import sys, torch; sys.path.insert(0, '$GRAFT_REPO_ROOT')
from cdnaml.ops import kernels as K
from cdnaml.models.tree.engine import find_thresholds
X = torch.randn((100000000, 100), device='cuda')
thr, nthr = find_thresholds(X[:10000].double().cpu().numpy(), 100, 40, {})
t = torch.from_numpy(thr.astype('float32')).cuda(); nt = torch.from_numpy(nthr).cuda()
for _ in range(3): K.binize(X, t, nt)
torch.cuda.synchronize()
" > $O/r$r.log 2>&1 || { echo fail $r; tail -3 $O/r$r.log; exit 1; }
  echo "rpt=$r: $(grep binize2 $(find $O/r$r -name '*kernel_stats.csv') | cut -d, -f4)"
done
