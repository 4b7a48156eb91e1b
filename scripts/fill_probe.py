"""Which Python calls issue the large device fills of one headline-shape fit (per-rank 1.25e7 rows): wraps the
torch fill entry points and prints those of >= 1e7 elements with the calling frames."""
import sys
import traceback

import torch

sys.path.insert(0, ".")
import cdnaml  # noqa: E402
from cdnaml.models.regression import RandomForestRegressor  # noqa: E402
from cdnaml.utils.synthetic import regression_shard  # noqa: E402

spark = cdnaml.SparkSession.builder.getOrCreate()
n = int(1.25e7)
X, y, _ = regression_shard(n, 100, 42, 0, 1, "cuda")
df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
est = RandomForestRegressor(numTrees=20, maxDepth=5, maxBins=40, seed=42)
m = est.fit(df)
m.transform(df).count()
torch.cuda.synchronize()
hits = []


def wrap(owner, name):
    orig = getattr(owner, name)

    def w(*a, **k):
        out = orig(*a, **k)
        t = out if isinstance(out, torch.Tensor) else (a[0] if a and isinstance(a[0], torch.Tensor) else None)
        if t is not None and t.is_cuda and t.numel() >= 10_000_000:
            hits.append((name, tuple(t.shape), t.dtype, "".join(traceback.format_stack(limit=7)[:-1])))
        return out
    setattr(owner, name, w)


for nm in ("zeros", "full", "ones", "zeros_like", "full_like", "ones_like"):
    wrap(torch, nm)
for nm in ("fill_", "zero_"):
    wrap(torch.Tensor, nm)
m = est.fit(df)
out = m.transform(df)
out.count()
torch.cuda.synchronize()
for name, shape, dt, st in hits:
    print(f"== {name} {shape} {dt}\n{st}")
print(f"{len(hits)} large fills")
