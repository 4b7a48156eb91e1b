"""Timing probe: RandomForestRegressor depth 10 (and 8) at 1e7 x 100, 20 trees (fit only)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cdnaml  # noqa: E402
from cdnaml.models.regression import RandomForestRegressor  # noqa: E402
from cdnaml.utils.synthetic import regression_shard  # noqa: E402

spark = cdnaml.SparkSession.builder.getOrCreate()
X, y, _ = regression_shard(int(1e7), 100, 42, 0, 1, spark.device)
df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
for depth in (8, 10):
    rf = RandomForestRegressor(numTrees=20, maxDepth=depth, maxBins=40, seed=42)
    rf.fit(df)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(2):
        m = rf.fit(df)
    torch.cuda.synchronize()
    print(f"depth {depth}: {(time.perf_counter() - t) / 2 * 1e3:.1f} ms per fit, nodes {m.totalNumNodes}", flush=True)
