"""Host profile of the RF classifier CrossValidator config (bench_configs clf) at 1e7 x 100."""
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
from cdnaml.ml.classification import RandomForestClassifier  # noqa: E402
from cdnaml.ml.evaluation import BinaryClassificationEvaluator  # noqa: E402
from cdnaml.ml.tuning import CrossValidator, ParamGridBuilder  # noqa: E402

spark = cdnaml.SparkSession.builder.getOrCreate()
df, n = bc._data(spark, int(float(os.environ.get("ROWS", "1e7"))), 100, cls=True)
rf = RandomForestClassifier(maxBins=40, seed=42)
t = time.perf_counter()
m = rf.setMaxDepth(5).setNumTrees(10).fit(df)
torch.cuda.synchronize()
print(f"single fit (cold): {(time.perf_counter() - t) * 1e3:.1f} ms")
t = time.perf_counter()
m = rf.fit(df)
torch.cuda.synchronize()
print(f"single fit: {(time.perf_counter() - t) * 1e3:.1f} ms")
grid = ParamGridBuilder().addGrid(rf.maxDepth, [2, 5, 10]).addGrid(rf.numTrees, [10, 20, 100]).build()
cv = CrossValidator(estimator=rf, estimatorParamMaps=grid, evaluator=BinaryClassificationEvaluator(), numFolds=3,
                    seed=42)
cv.fit(df)  # warm
torch.cuda.synchronize()
pr = cProfile.Profile()
t = time.perf_counter()
pr.enable()
cv.fit(df)
torch.cuda.synchronize()
pr.disable()
print(f"cv: {(time.perf_counter() - t) * 1e3:.1f} ms")
st = pstats.Stats(pr)
st.sort_stats("cumtime").print_stats(45)
st.sort_stats("tottime").print_stats(25)
st.sort_stats("tottime").print_stats(25)
