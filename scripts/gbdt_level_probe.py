"""Per-level rows / launch time of the GBDT config's histogram calls (bench_configs.py gbdt shape: 1e8 x 100,
depth 8, 256 bins): wraps K.seg_hist / K.seg_hist_codes with device syncs (so the times include launch gaps) and
prints, for the last tree, rows histogrammed, built slots and milliseconds per level."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench_configs as BC  # noqa: E402
import cdnaml  # noqa: E402
from cdnaml.models.xgboost import XgboostRegressor  # noqa: E402
from cdnaml.ops import kernels as K  # noqa: E402

log = []


def wrap(name, fn, rows_of):
    def w(*a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn(*a, **k)
        torch.cuda.synchronize()
        log.append((name, rows_of(a, k), (time.perf_counter() - t0) * 1e3))
        return out
    return w


K.seg_hist = wrap("seg_hist", K.seg_hist, lambda a, k: int(np.asarray(a[7])[:, 1].sum()))
K.seg_hist_codes = wrap("seg_hist_codes", K.seg_hist_codes, lambda a, k: -1)
spark = cdnaml.SparkSession.builder.getOrCreate()
n = int(float(sys.argv[1])) if len(sys.argv) > 1 else int(1e8)
df, _ = BC._data(spark, n, 100)
est = XgboostRegressor(n_estimators=3, max_depth=8, learning_rate=0.1, max_bin=256, random_state=42)
est.fit(df)
per_tree = len(log) // 3
for name, rows, ms in log[-per_tree:]:
    print(f"{name:16s} rows {rows:>11d}  {ms:7.3f} ms")
