"""Host time of the level loop's histogram-side calls at the per-rank shape (1.25e7 rows): wall time of each
K.codes_compact / K.seg_hist / K.seg_hist_codes call, and of the pieces inside seg_hist (work planning, upload),
for the last of a few fits.  Prints one line per call."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cdnaml  # noqa: E402
from cdnaml.models.regression import RandomForestRegressor  # noqa: E402
from cdnaml.models.tree import engine  # noqa: E402
from cdnaml.ops import kernels as K  # noqa: E402
from cdnaml.utils.synthetic import regression_shard  # noqa: E402

log = []


def wrap(mod, name):
    f = getattr(mod, name)

    def g(*a, **k):
        t = time.perf_counter()
        r = f(*a, **k)
        log.append((name, (time.perf_counter() - t) * 1e6))
        return r
    setattr(mod, name, g)


for n in ("codes_compact", "seg_hist", "seg_hist_codes", "_fill_chunk", "_seg_work", "upload", "_codes_compact_w",
          "_seg_hist_rec", "split_scan", "split_decode", "partition_codes", "hist_assemble"):
    wrap(K, n)
engine.K = K
spark = cdnaml.SparkSession.builder.getOrCreate()
X, y, _ = regression_shard(int(1.25e7), 100, 42, 0, 1, spark.device)
df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
rf = RandomForestRegressor(numTrees=20, maxDepth=5, maxBins=40, seed=42)
for i in range(4):
    log.clear()
    m = rf.fit(df)
    torch.cuda.synchronize()
for name, us in log:
    print(f"{name:20s} {us:9.1f} us")
