"""Records per level of the headline forest (RF 20 trees, depth 5, 40 bins, 1e8 x 100): for every record
histogram launch (levels 2-4, seg_hist_lane10) the slots, the records and the distinct rows they gather -- the
cross-slot reuse a row-ordered schedule could serve from cache.  ROWS=<n> (default 1e8)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cdnaml  # noqa: E402
from cdnaml.ml.regression import RandomForestRegressor  # noqa: E402
from cdnaml.models.tree import engine  # noqa: E402
from cdnaml.utils.synthetic import regression_shard  # noqa: E402

rows = int(float(os.environ.get("ROWS", "1e8")))
spark = cdnaml.SparkSession.builder.getOrCreate()
X, y, _ = regression_shard(rows, 100, 42, 0, 1, spark.device)
df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
K = engine.K
orig = K.seg_hist
info = []


def spy(bins, d, B, perm, v0p, v1p, wp, segs, S, *a, **k):
    if k.get("rec"):
        segs_ = segs.reshape(-1, 3)
        total = int(segs_[:, 1].sum())
        r = perm[:total] & 0x7FFFFFFF
        uniq = int(torch.unique(r).numel())
        info.append((S, total, uniq))
    return orig(bins, d, B, perm, v0p, v1p, wp, segs, S, *a, **k)


K.seg_hist = spy
rf = RandomForestRegressor(numTrees=20, maxDepth=5, maxBins=40, seed=42)
rf.fit(df)
torch.cuda.synchronize()
for S, total, uniq in info:
    print(f"slots {S:4d} records {total:.3e} distinct rows {uniq:.3e} reuse {total / max(uniq, 1):.2f} "
          f"density/slot {total / S / rows:.4f}", flush=True)
