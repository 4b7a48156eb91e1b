"""Host time at the end of a fit (per-rank 1.25e7 shape): from the last level's decisions reaching the host to
the transform's predict launch, the GPU idles.  Wraps the pieces in perf_counter timers and prints the split."""
import os
import sys
import time
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cdnaml  # noqa: E402
from cdnaml.models.regression import RandomForestRegressor  # noqa: E402
from cdnaml.models.tree import engine  # noqa: E402
from cdnaml.ops import kernels as K  # noqa: E402
from cdnaml.utils.synthetic import regression_shard  # noqa: E402

T = defaultdict(float)
marks = {}


def wrap(obj, name, key):
    f = getattr(obj, name)

    def g(*a, **k):
        t = time.perf_counter()
        r = f(*a, **k)
        T[key] += time.perf_counter() - t
        marks[key + ".end"] = time.perf_counter()
        marks[key + ".sync"] = marks.get("sync", 0.0)  # the last device wait inside the call
        return r
    setattr(obj, name, g)


wrap(engine.ForestTrainer, "train", "train")
# the last device -> host wait inside train(): the final level's decisions arriving
_cpu, _evs = torch.Tensor.cpu, torch.cuda.Event.synchronize


def _cpu_w(self, *a, **k):
    r = _cpu(self, *a, **k)
    marks["sync"] = time.perf_counter()
    return r


def _evs_w(self):
    r = _evs(self)
    marks["sync"] = time.perf_counter()
    return r


torch.Tensor.cpu = _cpu_w
torch.cuda.Event.synchronize = _evs_w
wrap(engine.Forest, "heap_arrays", "heap_arrays")
wrap(K, "tree_predict_heap", "predict_launch")
orig_pred = K.tree_predict_heap


rows = int(float(os.environ.get("ROWS", "1.25e7")))
spark = cdnaml.SparkSession.builder.getOrCreate()
X, y, _ = regression_shard(rows, 100, 42, 0, 1, spark.device)
df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
rf = RandomForestRegressor(labelCol="label", featuresCol="features", numTrees=20, maxDepth=5, maxBins=40, seed=42)
tail = []
for i in range(8):
    t0 = time.perf_counter()
    m = rf.fit(df)
    t1 = time.perf_counter()
    out = m.transform(df)
    t2 = time.perf_counter()
    out._plan.execute()
    t3 = time.perf_counter()
    torch.cuda.synchronize() if torch.cuda.is_available() else None
    if i >= 3:
        tail.append((marks["train.end"] - marks["train.sync"], t1 - marks["train.end"], t2 - t1, t3 - t2))
for z, a, b, c in tail:
    print(f"train() after its last sync: {z * 1e3:.3f} ms  fit after train(): {a * 1e3:.3f} ms  "
          f"transform(): {b * 1e3:.3f} ms  execute(): {c * 1e3:.3f} ms")
import cProfile, pstats  # noqa: E401,E402
pr = cProfile.Profile()
m = rf.fit(df)
torch.cuda.synchronize() if torch.cuda.is_available() else None
pr.enable()
out = m.transform(df)
out._plan.execute()
pr.disable()
pstats.Stats(pr).sort_stats("cumtime").print_stats(25)
# whole fit + transform, Python self time (what the host does while the GPU may idle)
pr = cProfile.Profile()
torch.cuda.synchronize() if torch.cuda.is_available() else None
pr.enable()
m = rf.fit(df)
m.transform(df)._plan.execute()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
