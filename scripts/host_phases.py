"""Host wall time of each level phase of the tree trainer (ForestTrainer._level_* methods) for the last of a few
fits at the per-rank shape (ROWS, default 1.25e7): where the host spends the time between a level's decisions and
the next level's first launch (the GPU idles through whatever exceeds the queued partition)."""
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


def wrap(cls, name):
    f = getattr(cls, name)

    def g(*a, **k):
        t = time.perf_counter()
        r = f(*a, **k)
        log.append((name, t, time.perf_counter()))
        return r
    setattr(cls, name, g)


for n in ("_level_tables", "_level_histogram", "_level_reduce", "_level_decide", "_level_advance", "_fit_paths",
          "_fit_rows", "_fit_finish"):
    wrap(engine.ForestTrainer, n)
for n in ("seg_hist_codes", "codes_compact", "seg_hist", "partition_codes", "split_decode", "split_scan",
          "_codes_compact_w", "_seg_hist_rec", "upload"):
    wrap(K, n)
_ev_sync = torch.cuda.Event.synchronize


SPIN = os.environ.get("SPIN", "0") == "1"


def _sync(self):
    t = time.perf_counter()
    if SPIN:
        while not self.query():
            pass
    else:
        _ev_sync(self)
    log.append(("event.synchronize", t, time.perf_counter()))


torch.cuda.Event.synchronize = _sync

rows = int(float(os.environ.get("ROWS", "1.25e7")))
spark = cdnaml.SparkSession.builder.getOrCreate()
X, y, _ = regression_shard(rows, 100, 42, 0, 1, spark.device)
df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
rf = RandomForestRegressor(labelCol="label", featuresCol="features", numTrees=20, maxDepth=5, maxBins=40, seed=42)
for _ in range(3):
    log.clear()
    t0 = time.perf_counter()
    rf.fit(df)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
print(f"fit wall {1e3 * (t1 - t0):.2f} ms (SPIN={int(SPIN)})")
for name, a, b in log:
    print(f"{1e6 * (a - t0):9.1f} us +{1e6 * (b - a):8.1f} us  {name}")
