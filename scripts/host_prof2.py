"""Host time of the transform that follows a fit (the GPU idles through it at the end of every bench step):
cProfile of model.transform(df)._plan.execute() only, after the fit's queue has drained."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cdnaml  # noqa: E402
from cdnaml.models.regression import RandomForestRegressor  # noqa: E402
from cdnaml.utils.synthetic import regression_shard  # noqa: E402

spark = cdnaml.SparkSession.builder.getOrCreate()
X, y, _ = regression_shard(int(1.25e7), 100, 42, 0, 1, spark.device)
df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
rf = RandomForestRegressor(labelCol="label", featuresCol="features", numTrees=20, maxDepth=5, maxBins=40, seed=42)
pr = cProfile.Profile()
for i in range(4):
    t0 = time.perf_counter()
    m = rf.fit(df)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    if i >= 1:
        pr.enable()
    out = m.transform(df)._plan.execute()
    t3 = time.perf_counter()
    if i >= 1:
        pr.disable()
    torch.cuda.synchronize()
    print(f"fit host {1e3 * (t1 - t0):.2f} ms, drain {1e3 * (t2 - t1):.2f} ms, transform host {1e3 * (t3 - t2):.2f} ms")
pstats.Stats(pr).sort_stats("cumtime").print_stats(40)
