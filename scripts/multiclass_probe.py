"""Timing probe: RandomForestClassifier fit, 20 trees, depth 5, 40 bins, binary vs 3-class labels (the 3-class
fit must take the packed record path -- K.cls3_expand once per level -- at every row count).
ROWS=<n> (default 1e7); 1e8 x 100 is VERDICT r5 item 6's shape."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cdnaml  # noqa: E402
from cdnaml.ml.classification import RandomForestClassifier  # noqa: E402
from cdnaml.models.tree import engine  # noqa: E402
from cdnaml.utils.synthetic import regression_shard  # noqa: E402

rows = int(float(os.environ.get("ROWS", "1e7")))
spark = cdnaml.SparkSession.builder.getOrCreate()
X, y, _ = regression_shard(rows, 100, 42, 0, 1, spark.device)
q = torch.quantile(y[:100000].float(), torch.tensor([1 / 3, 2 / 3], device=y.device))
calls = {"n": 0}
orig = engine.K.cls3_expand


def counted(*a, **k):
    calls["n"] += 1
    return orig(*a, **k)


engine.K.cls3_expand = counted
res = {}
for name, lab in [("binary", (y > q[0]).double()), ("3-class", (y > q[0]).double() + (y > q[1]).double())]:
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": lab})
    est = RandomForestClassifier(numTrees=20, maxDepth=5, maxBins=40, seed=42)
    est.fit(df)
    torch.cuda.synchronize()
    ts = []
    calls["n"] = 0
    for _ in range(3):
        t = time.perf_counter()
        est.fit(df)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    res[name] = min(ts)
    print(f"{name}: rows={rows:.2e} {' '.join(f'{x:.1f}' for x in ts)} ms per fit; packed 3-class levels "
          f"{calls['n'] / 3:.0f} per fit", flush=True)
print(f"3-class / binary = {res['3-class'] / res['binary']:.3f}", flush=True)
