"""Boosting margins updated by the level partitions (engine.train(margin=...), hist5.hip partition5 margin
mode + split.hip split_decode leaf values) against the tree walk after each round (predict_binned_add): the F
updates are the same fp32 operations, so every later round's gradients -- and the whole boosted forest -- must be
bit-identical."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("depth,bins,missing", [(8, 256, True), (5, 64, False), (3, 256, False)])
def test_partition_margins_equal_tree_walk(monkeypatch, depth, bins, missing):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import cdnaml
    from cdnaml.models.tree import engine
    from cdnaml.models.xgboost import XgboostRegressor
    from cdnaml.utils.synthetic import forest_digest
    spark = cdnaml.SparkSession.builder.getOrCreate()
    g = torch.Generator(device="cuda").manual_seed(depth)
    n = 200_003
    X = torch.randn((n, 30), generator=g, device="cuda")
    if missing:
        X[::9, 4] = float("nan")
    y = (X[:, 0].nan_to_num() * 2 + torch.sin(X[:, 1] * 3) + (X[:, 2] > 0.3).float()).double()
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
    calls = {"applied": 0}
    orig = engine.ForestTrainer.train

    def counted(self, *a, **k):
        out = orig(self, *a, **k)
        calls["applied"] += int(getattr(self, "margin_applied", False))
        return out
    monkeypatch.setattr(engine.ForestTrainer, "train", counted)
    est = XgboostRegressor(n_estimators=12, max_depth=depth, max_bin=bins, learning_rate=0.3)
    monkeypatch.setattr(engine, "GBDT_MARGIN", True)
    m1 = est.fit(df)
    assert calls["applied"] == 12  # every round took the partition margins
    calls["applied"] = 0
    monkeypatch.setattr(engine, "GBDT_MARGIN", False)
    m0 = est.fit(df)
    assert calls["applied"] == 0
    assert forest_digest(m1._forest) == forest_digest(m0._forest)
    p1 = m1.transform(df).select("prediction").toPandas()["prediction"].to_numpy()
    p0 = m0.transform(df).select("prediction").toPandas()["prediction"].to_numpy()
    assert np.array_equal(p1, p0)
