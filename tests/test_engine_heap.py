"""The predict heap table filled by ForestTrainer.train level by level equals Forest.heap_arrays' table built from
the finished forest (tree of every node, heap slot from the root path, leaf values and thresholds as fp32 bits);
and the vectorised Forest.set_splits equals the per-node assignment."""
import numpy as np
import torch

from cdnaml.models.tree.engine import Forest
from cdnaml.ops import kernels as K


def test_trainer_heap_equals_forest_walk():
    import cdnaml
    from cdnaml.models.regression import RandomForestRegressor
    spark = cdnaml.SparkSession.builder.getOrCreate()
    g = torch.Generator().manual_seed(0)
    for n, d, T, depth in ((3000, 6, 5, 4), (2000, 12, 7, 6), (500, 4, 3, 8)):
        X = torch.randn(n, d, generator=g)
        y = (X[:, 0] * 2 - X[:, 1] + torch.sin(X[:, 2])).double()
        df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
        f = RandomForestRegressor(numTrees=T, maxDepth=depth, maxBins=16, seed=1, minInstancesPerNode=3).fit(df)._forest
        f.settle()  # a deferred last level fills the host arrays when it runs (test_device_last_level_heap)
        assert f._heap_np is not None
        pre = f._heap_np
        f._heap_np = None
        st, vals, D, _ = f.heap_struct()
        assert D == pre[2]
        np.testing.assert_array_equal(st, pre[0])
        # the trainer's per-slot values hold every node's value (splits too); the packed table reads leaves only
        np.testing.assert_array_equal(K.pack_heap(st, vals, D), K.pack_heap(pre[0], pre[1], pre[2]))


def test_device_last_level_heap(spark):
    """The last split level decided on the device (K.heap_last_level into a copy of the packed heap, the host side
    left pending): the device table equals the host arrays' table once the pending work has run, the forest
    (digest) equals the one grown with the deferral off, and so do the predictions (cpu and, marked gpu, cuda:
    there the HIP kernel writes the table and the predictor reads it before the host has seen the level)."""
    from cdnaml.models.regression import RandomForestRegressor
    from cdnaml.models.tree import engine as E
    from cdnaml.utils.synthetic import forest_digest
    g = torch.Generator().manual_seed(5)
    X = torch.randn(4000, 9, generator=g)
    y = (X[:, 0] * 2 - X[:, 1] + torch.sin(X[:, 2]) + 0.2 * torch.randn(4000, generator=g)).double()
    df = spark.createDataFrameFromLocalTensors({"features": X.to(spark.device), "label": y.to(spark.device)})
    est = RandomForestRegressor(numTrees=6, maxDepth=5, maxBins=24, seed=2, minInstancesPerNode=2)
    m = est.fit(df)
    f = m._forest
    key = ("heap", str(spark.device), "value")
    assert key in f._dev and f._pending, "the last level was not deferred"
    h_dev, D, _ = f._dev[key]
    p1 = m.transform(df).select("prediction").toPandas()["prediction"].to_numpy()
    assert not f._pending  # the predictor ran the pending level right after its launch
    pre = f._heap_np
    assert pre is not None and pre[2] == D == 5
    np.testing.assert_array_equal(h_dev.cpu().numpy(), K.pack_heap(*pre))
    old = E.HEAP_LAST_DEVICE
    try:
        E.HEAP_LAST_DEVICE = False
        m2 = est.fit(df)
    finally:
        E.HEAP_LAST_DEVICE = old
    f2 = m2._forest
    assert key not in f2._dev and forest_digest(f2) == forest_digest(f)
    p2 = m2.transform(df).select("prediction").toPandas()["prediction"].to_numpy()
    np.testing.assert_array_equal(p1, p2)


def test_set_splits_vectorised():
    rng = np.random.default_rng(0)
    f = Forest(1)
    f.add_many(np.zeros((50, 1)), np.ones(50), 0, np.zeros(50))
    fids = np.sort(rng.choice(np.arange(10, 40), 12, replace=False))
    feats, gains = rng.integers(0, 9, 12), rng.random(12)
    bins, thrs, has = rng.integers(0, 30, 12), rng.random(12), rng.random(12) < 0.7
    lefts, rights = rng.integers(50, 99, 12), rng.integers(50, 99, 12)
    f.set_splits(fids, feats, gains, bins, thrs, has, lefts, rights)
    for j, a in enumerate(fids):
        assert f.feat[a] == feats[j] and f.gain[a] == gains[j] and f.left[a] == lefts[j] and f.right[a] == rights[j]
        assert f.bin[a] == (bins[j] if has[j] else 0) and f.thr[a] == (thrs[j] if has[j] else 0.0)
        assert type(f.feat[a]) is int and type(f.thr[a]) is float
    other = np.setdiff1d(np.arange(50), fids)
    assert all(f.feat[a] == -1 and f.left[a] == -1 for a in other)


def test_last_level_bookkeeping_settles_on_first_read():
    """ForestTrainer.train leaves the last level's node-list bookkeeping with the forest (run by the predictor
    right after its launch, or by the first reader): readers always see the complete forest, copies settle."""
    import copy
    import torch
    import cdnaml
    from cdnaml.models.regression import RandomForestRegressor
    from cdnaml.utils.synthetic import forest_digest
    spark = cdnaml.SparkSession.builder.getOrCreate()
    g = torch.Generator().manual_seed(3)
    X = torch.randn((3000, 8), generator=g)
    y = (X[:, 0] * 2 + X[:, 1]).double()
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
    m = RandomForestRegressor(numTrees=3, maxDepth=4, seed=1).fit(df)
    f = m._forest
    assert f._pending  # deferred past fit
    c = copy.deepcopy(f)  # a copy settles the original first and carries no pending work
    assert not f._pending and not c._pending
    assert forest_digest(c) == forest_digest(f)
    m2 = RandomForestRegressor(numTrees=3, maxDepth=4, seed=1).fit(df)
    assert m2._forest._pending
    n = len(m2._forest.feat)  # any node-list read settles
    assert not m2._forest._pending and n == len(f.feat)
    assert forest_digest(m2._forest) == forest_digest(f)
