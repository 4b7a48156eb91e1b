"""Host time of LinearRegression.fit at the config-2 shape (1e7 x 100, bf16 Gram): cProfile over 20 fits."""
import cProfile
import pstats
import sys
import time

import torch

sys.path.insert(0, ".")
import bench_configs as BC  # noqa: E402
import cdnaml  # noqa: E402
from cdnaml.models.regression import LinearRegression  # noqa: E402

spark = cdnaml.SparkSession.builder.getOrCreate()
df, n = BC._data(spark, int(1e7), 100)
lr = LinearRegression(gramPrecision="bf16")
for _ in range(3):
    lr.fit(df)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    lr.fit(df)
torch.cuda.synchronize()
print(f"fit {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms")
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    lr.fit(df)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(35)
