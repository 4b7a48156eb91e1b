"""Timing probe: regression trees deeper than 8 levels at 1e7 x 100 (fit only; A/B with CDNAML_DEEP_REG)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cdnaml  # noqa: E402
from cdnaml.models.regression import DecisionTreeRegressor, RandomForestRegressor  # noqa: E402
from cdnaml.utils.synthetic import regression_shard  # noqa: E402

spark = cdnaml.SparkSession.builder.getOrCreate()
X, y, _ = regression_shard(int(1e7), 100, 42, 0, 1, spark.device)
df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
tag = os.environ.get("CDNAML_DEEP_REG", "1")
for name, est in [("rf20 depth 8", RandomForestRegressor(numTrees=20, maxDepth=8, maxBins=40, seed=42)),
                  ("rf20 depth 10", RandomForestRegressor(numTrees=20, maxDepth=10, maxBins=40, seed=42)),
                  ("dt depth 12", DecisionTreeRegressor(maxDepth=12, maxBins=40, seed=42))]:
    if len(sys.argv) > 1 and sys.argv[1] not in name:
        continue
    est.fit(df)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(2):
        m = est.fit(df)
    torch.cuda.synchronize()
    print(f"DEEP_REG={tag} {name}: {(time.perf_counter() - t) / 2 * 1e3:.1f} ms per fit", flush=True)
