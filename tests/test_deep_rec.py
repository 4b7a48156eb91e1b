"""Binary classification forests deeper than the u16 row codes (levels >= 8 on node ids): the record histograms
continue through K.node_compact (seg.hip node_compact_kernel) instead of the node-id histogram kernel; the forests
must be bit-identical either way (class counts are exact integers on both paths)."""
import numpy as np
import pytest
import torch


def _devices():
    return ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("device", _devices())
@pytest.mark.parametrize("depth,trees", [(10, 6), (11, 3)])
def test_deep_record_histograms_equal_node_id_kernel(device, depth, trees, monkeypatch):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    import cdnaml
    from cdnaml.models.tree import engine
    from cdnaml.ml.classification import RandomForestClassifier
    from cdnaml.utils.synthetic import forest_digest
    from tests.conftest import session_device
    with session_device(device):
        spark = cdnaml.SparkSession.builder.getOrCreate()
        g = torch.Generator().manual_seed(depth)
        n = 60_000 if device == "cpu" else 400_000
        X = torch.randn((n, 12), generator=g)
        logit = X[:, 0] * 2 - X[:, 1] + torch.sin(3 * X[:, 2]) + 0.5 * X[:, 3] * X[:, 4]
        y = (logit + 0.3 * torch.randn(n, generator=g) > 0).double()
        df = spark.createDataFrameFromLocalTensors({"features": X.to(device), "label": y.to(device)})
        est = RandomForestClassifier(numTrees=trees, maxDepth=depth, maxBins=32, seed=5)
        calls = {"n": 0}
        orig = engine.K.node_compact

        def counted(*a, **k):
            calls["n"] += 1
            return orig(*a, **k)
        monkeypatch.setattr(engine.K, "node_compact", counted)
        digests = []
        try:
            for cap in (engine.K.NODE_COMPACT_MAX_LOC, 0):
                # cap 0: every deep level takes the node-id histogram kernels instead of the node-id records
                monkeypatch.setattr(engine.K, "NODE_COMPACT_MAX_LOC", cap)
                digests.append(forest_digest(est.fit(df)._forest))
        finally:
            spark.stop()
        assert calls["n"] >= 1  # the deep levels took the record path
        assert digests[0] == digests[1]


@pytest.mark.parametrize("device", _devices())
@pytest.mark.parametrize("est_kind,depth,trees", [("rf", 10, 4), ("rf", 11, 2)])
def test_deep_regression_prefix_is_depth8_forest(device, est_kind, depth, trees, monkeypatch):
    """Regression forests deeper than 8 (engine.DEEP_REG): the record levels down to 8, then node ids + record histograms.
    The depth-8 prefix of the deep forest is bit-identical to the depth-8 forest, and the deep levels improve the
    training fit."""
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    import cdnaml
    from cdnaml.models.tree import engine
    from cdnaml.models.tree.fused import truncate_forest
    from cdnaml.ml.regression import DecisionTreeRegressor, RandomForestRegressor
    from cdnaml.utils.synthetic import forest_digest
    from tests.conftest import session_device
    with session_device(device):
        spark = cdnaml.SparkSession.builder.getOrCreate()
        g = torch.Generator().manual_seed(depth)
        n = 50_000 if device == "cpu" else 300_000
        X = torch.randn((n, 10), generator=g)
        y = (3 * X[:, 0] - X[:, 1] + torch.sin(4 * X[:, 2]) + X[:, 3] * X[:, 4]
             + 0.2 * torch.randn(n, generator=g)).double()
        df = spark.createDataFrameFromLocalTensors({"features": X.to(device), "label": y.to(device)})
        calls = {"n": 0}
        orig = engine.K.node_compact

        def counted(*a, **k):
            calls["n"] += 1
            return orig(*a, **k)
        monkeypatch.setattr(engine.K, "node_compact", counted)

        def est(D):
            if est_kind == "rf":
                return RandomForestRegressor(numTrees=trees, maxDepth=D, maxBins=32, seed=3)
            return DecisionTreeRegressor(maxDepth=D, maxBins=32, seed=3)
        try:
            deep = est(depth).fit(df)
            assert calls["n"] >= 1  # the levels below 8 built record histograms from node ids
            shallow = est(8).fit(df)
            cut = truncate_forest(deep._forest, trees, 8)
            assert forest_digest(cut) == forest_digest(shallow._forest)

            def mse(m):
                p = m.transform(df).select("prediction").toPandas()["prediction"].to_numpy()
                return float(((p - y.numpy()) ** 2).mean())
            assert mse(deep) < mse(shallow)
        finally:
            spark.stop()


@pytest.mark.parametrize("device", _devices())
def test_deep_fallback_node_histograms_use_bootstrap_weights(device, monkeypatch):
    """Past NODE_COMPACT_MAX_LOC active nodes per tree the deep levels fall back to the node-id histogram kernel,
    which reads the row weights: with the bootstrap draws written straight as row codes (GPU BootstrapCodes, no
    weights tensor) they must come from the decoded codes -- the forest equals the one grown from the same draws
    passed as a weights tensor (K.POISSON_CODES off)."""
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    import cdnaml
    from cdnaml.models.tree import engine
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.utils.synthetic import forest_digest
    from tests.conftest import session_device
    with session_device(device):
        spark = cdnaml.SparkSession.builder.getOrCreate()
        g = torch.Generator().manual_seed(17)
        n = 40_000 if device == "cpu" else 200_000
        X = torch.randn((n, 10), generator=g)
        y = (2 * X[:, 0] + torch.sin(3 * X[:, 1]) + 0.3 * torch.randn(n, generator=g)).double()
        df = spark.createDataFrameFromLocalTensors({"features": X.to(device), "label": y.to(device)})
        est = RandomForestRegressor(numTrees=3, maxDepth=10, maxBins=32, seed=2)
        monkeypatch.setattr(engine.K, "NODE_COMPACT_MAX_LOC", 1)
        try:
            got = {}
            for codes in (True, False):
                monkeypatch.setattr(engine.K, "POISSON_CODES", codes)
                got[codes] = forest_digest(est.fit(df)._forest)
        finally:
            spark.stop()
        assert got[True] == got[False]


def test_cut_forest_lists_are_frozen(spark):
    """a forest cut by the fused tuner is immutable after the cut (in-place mutation of its node fields
    raises); pickling and reassigning a field still work."""
    import pickle
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.models.tree.fused import truncate_forest
    from cdnaml.utils.synthetic import forest_digest
    g = torch.Generator().manual_seed(0)
    X = torch.randn((3000, 6), generator=g)
    y = (X[:, 0] - 2 * X[:, 1]).double()
    df = spark.createDataFrameFromLocalTensors({"features": X.to(spark.device), "label": y.to(spark.device)})
    m = RandomForestRegressor(numTrees=3, maxDepth=4, maxBins=16, seed=1).fit(df)
    cut = truncate_forest(m._forest, 2, 3)
    for op in (lambda: cut.thr.__setitem__(0, 1.0), lambda: cut.feat.append(-1), lambda: cut.value.pop(),
               lambda: cut.roots.extend([0])):
        with pytest.raises(TypeError):
            op()
    back = pickle.loads(pickle.dumps(cut))
    assert forest_digest(back) == forest_digest(cut)
    with pytest.raises(TypeError):
        back.thr[0] = 1.0
    d0 = forest_digest(cut)
    cut.thr = [t + 0.0 for t in cut.thr]
    cut.thr[0] = cut.thr[0]
    assert forest_digest(cut) == d0
