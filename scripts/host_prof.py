"""Host-side profile of the headline step at the per-rank shape of the 8-GPU point (1.25e7 rows): cProfile over 3
steps after 2 warmups, top functions by own time.  Shows the Python/numpy work between a level's decisions and
the next level's launches (the GPU idles through it)."""
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

rows = int(float(os.environ.get("ROWS", "1.25e7")))
spark = cdnaml.SparkSession.builder.getOrCreate()
X, y, _ = regression_shard(rows, 100, 42, 0, 1, spark.device)
df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
rf = RandomForestRegressor(labelCol="label", featuresCol="features", numTrees=20, maxDepth=5, maxBins=40, seed=42)


def step():
    m = rf.fit(df)
    m.transform(df)._plan.execute()


for _ in range(2):
    step()
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for _ in range(3):
    step()
torch.cuda.synchronize()
pr.disable()
print(f"3 steps: {(time.perf_counter() - t0) * 1e3:.1f} ms")
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)
st.print_callers(r"method 'to' of|method 'cpu' of|method 'item' of|Event.synchronize")
