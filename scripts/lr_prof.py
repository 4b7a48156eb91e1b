"""Where the LinearRegression fit's time goes off the Gram kernel (config 2 shape: 1e7 x 100, bf16 Gram):
cProfile of 20 fits after warmup, plus the wall time per fit."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = [sys.argv[0]]
import bench_configs as bc  # noqa: E402
import cdnaml  # noqa: E402
from cdnaml.models.regression import LinearRegression  # noqa: E402

spark = cdnaml.SparkSession.builder.getOrCreate()
df, n = bc._data(spark, int(1e7), 100)
lr = LinearRegression(gramPrecision="bf16")
for _ in range(5):
    lr.fit(df)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(20):
    lr.fit(df)
torch.cuda.synchronize()
print(f"fit: {(time.perf_counter() - t) / 20 * 1e3:.3f} ms")
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    lr.fit(df)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
