"""Timing probe: regression trees deeper than 8 levels at 1e7 x 100 (fit only; A/B with CDNAML_DEEP_REG)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cdnaml  # noqa: E402
from cdnaml.models.regression import DecisionTreeRegressor, RandomForestRegressor  # noqa: E402
from cdnaml.utils.synthetic import regression_shard  # noqa: E402

if os.environ.get("GC_OFF") == "1":
    import gc
    gc.disable()
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
    ts = []
    for _ in range(int(os.environ.get("REPS", "5"))):
        t = time.perf_counter()
        m = est.fit(df)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
        del m
    print(f"DEEP_REG={tag} {name}: median {sorted(ts)[len(ts) // 2]:.1f} ms per fit "
          f"({' '.join(f'{x:.1f}' for x in ts)})", flush=True)
