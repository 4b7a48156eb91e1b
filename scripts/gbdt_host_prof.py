"""Host profile of boosting rounds (bench_configs gbdt shape, fewer trees): where the level loop's host time goes
(the GPU idles between a level's decisions and the next level's uploads while the host plans)."""
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
from cdnaml.models.xgboost import XgboostRegressor  # noqa: E402

spark = cdnaml.SparkSession.builder.getOrCreate()
df, n = bc._data(spark, int(float(os.environ.get("ROWS", "1e8"))), 100)
trees = int(os.environ.get("TREES", "40"))
est = XgboostRegressor(n_estimators=trees, max_depth=8, learning_rate=0.1, max_bin=256, random_state=42)
est.fit(df)
torch.cuda.synchronize()
pr = cProfile.Profile()
t = time.perf_counter()
pr.enable()
est.fit(df)
torch.cuda.synchronize()
pr.disable()
ms = (time.perf_counter() - t) * 1e3
print(f"fit: {ms:.1f} ms = {ms / trees:.2f} ms/tree", flush=True)
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumulative").print_stats(40)
