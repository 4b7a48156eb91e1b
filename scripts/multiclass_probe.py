"""Timing probe: RandomForestClassifier fit at 1e7 x 100, 20 trees, depth 5, binary vs 3-class labels."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cdnaml  # noqa: E402
from cdnaml.ml.classification import RandomForestClassifier  # noqa: E402
from cdnaml.utils.synthetic import regression_shard  # noqa: E402

spark = cdnaml.SparkSession.builder.getOrCreate()
X, y, _ = regression_shard(int(1e7), 100, 42, 0, 1, spark.device)
q = torch.quantile(y[:100000].float(), torch.tensor([1 / 3, 2 / 3], device=y.device))
for name, lab in [("binary", (y > q[0]).double()), ("3-class", (y > q[0]).double() + (y > q[1]).double())]:
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": lab})
    est = RandomForestClassifier(numTrees=20, maxDepth=5, maxBins=40, seed=42)
    est.fit(df)
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        est.fit(df)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    print(f"{name}: {' '.join(f'{x:.1f}' for x in ts)} ms per fit", flush=True)
