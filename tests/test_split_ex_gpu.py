"""K6 for classification and categorical features (split.hip split_scan_ex_kernel) against the torch split chain it
replaces (ForestTrainer._best_splits): same feature, position, child statistics and category sets; whole forests
(ML 06 categoricals, L07 RandomForestClassifier) equal the torch-path forests."""
import numpy as np
import pytest
import torch

from cdnaml.ops import _lib, kernels as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _lib.lib()
    return torch.device("cuda:0")


def _trainer(kind, C, nthr, categorical, min_inst=1.0):
    from cdnaml.models.tree.engine import ForestTrainer, TreeParams
    tr = object.__new__(ForestTrainer)
    tr.p = TreeParams(impurity=kind, num_classes=C, min_instances=min_inst)
    tr.classification = kind in ("gini", "entropy")
    tr.C = C if tr.classification else 0
    tr.stats_k = C if tr.classification else 2

    class _D:
        pass
    tr.data = _D()
    tr.data.nthr = nthr
    tr.data.categorical = categorical
    tr.data.missing_bin = False
    return tr


@pytest.mark.parametrize("kind,C", [("gini", 2), ("gini", 5), ("entropy", 3), ("variance", 2)])
def test_split_scan_ex_matches_torch(dev, kind, C):
    rng = np.random.default_rng(C + len(kind))
    A, d, B = 24, 12, 40
    cat = {1: 7, 4: 33, 9: 40}
    nthr = np.full(d, B - 1, dtype=np.int32)
    nthr[[3, 7]] = [10, 25]
    for f in cat:
        nthr[f] = -1
    if kind == "variance":
        W = rng.integers(0, 30, size=(A, d, B)).astype(np.float64)
        S = np.round(rng.normal(size=(A, d, B)) * W * 64) / 64  # exact multiples of 2^-6
        H = np.stack([W, S], -1)
    else:
        H = rng.integers(0, 12, size=(A, d, B, C)).astype(np.float64)
    H[:, :, 35:] = 0                       # empty tail bins
    H[3, 4, :] = 0
    H[3, 4, 5] = [9.0] + [0.0] * (H.shape[-1] - 1)   # a categorical feature with one non-empty category
    tr = _trainer(kind, C, nthr, cat)
    Ht = torch.from_numpy(H).to(dev)
    words = rng.integers(0, 2 ** 32, size=(A, 1), dtype=np.uint64).astype(np.uint32) | np.uint32(0b1000010010)
    masks = torch.from_numpy(words.view(np.int32)).to(dev)
    for mk in (None, masks):
        tot = tr._node_stats(Ht, None)
        gain, bf, bb, lst, rst, order, cat_feats, _ = tr._best_splits(Ht, tot, mk)
        so, tot2, cm = K.split_scan_ex(Ht, torch.from_numpy(nthr).to(dev), mk, kind, 1.0)
        kk = tot.shape[1]
        ok = torch.isfinite(gain).cpu()
        assert torch.equal(ok, torch.isfinite(so[:, 0]).cpu())
        assert torch.equal(tot.cpu(), tot2.cpu())
        assert torch.equal(bf.cpu()[ok].double(), so[:, 1].cpu()[ok])
        assert torch.equal(bb.cpu()[ok].double(), so[:, 2].cpu()[ok])
        torch.testing.assert_close(so[:, 0].cpu()[ok], gain.cpu()[ok], rtol=1e-13, atol=0)
        assert torch.equal(so[:, 4:4 + kk].cpu()[ok], lst.cpu()[ok])
        assert torch.equal(so[:, 4 + kk:4 + 2 * kk].cpu()[ok], rst.cpu()[ok])
        oh = order.cpu().numpy()
        cmh = (cm.cpu().numpy().astype(np.int64) & 0xFFFFFFFF).astype(np.uint32)
        for a in np.nonzero(ok.numpy())[0]:
            f, b = int(bf[a]), int(bb[a])
            if f in cat:
                m = np.zeros(8, dtype=np.uint32)
                for c in oh[a, cat_feats.index(f), :b + 1]:
                    m[int(c) >> 5] |= np.uint32(1) << np.uint32(int(c) & 31)
                assert np.array_equal(m, cmh[a]), (a, f, b)


@pytest.mark.parametrize("flow", ["ml06_categorical_dt", "l07_rf_classifier"])
def test_forests_native_ex_equal_torch_path(dev, flow, monkeypatch):
    import cdnaml
    from cdnaml.models.tree import engine
    from cdnaml.utils.synthetic import forest_digest
    import pandas as pd
    spark = cdnaml.SparkSession.builder.getOrCreate()
    rng = np.random.default_rng(11)
    n = 40_000
    pdf = pd.DataFrame({"hood": [f"h{i}" for i in rng.integers(0, 37, n)],
                        "room": rng.choice(["entire", "private", "shared", "hotel"], n),
                        "beds": rng.integers(1, 6, n).astype(float), "lat": rng.normal(size=n),
                        "lon": rng.normal(size=n)})
    hood_num = pdf.hood.str[1:].astype(int)
    price = 40 * pdf.beds + 15 * (hood_num % 5) + 60 * (pdf.room == "entire") + 10 * pdf.lat + rng.normal(size=n) * 5
    from cdnaml.ml.feature import StringIndexer, VectorAssembler
    from cdnaml.ml.classification import RandomForestClassifier
    from cdnaml.ml.regression import DecisionTreeRegressor
    pdf["label"] = price if flow == "ml06_categorical_dt" else \
        np.digitize(price, np.quantile(price, [0.3, 0.7])).astype(float)
    sdf = spark.createDataFrame(pdf)
    # ML 06:42-63: StringIndexer'd categoricals carry nominal metadata through the VectorAssembler
    sdf = StringIndexer(inputCols=["hood", "room"], outputCols=["hoodIdx", "roomIdx"]).fit(sdf).transform(sdf)
    df = VectorAssembler(inputCols=["hoodIdx", "roomIdx", "beds", "lat", "lon"], outputCol="features").transform(sdf)
    if flow == "ml06_categorical_dt":
        est = DecisionTreeRegressor(maxDepth=6, maxBins=40)
    else:
        est = RandomForestClassifier(numTrees=10, maxDepth=6, maxBins=40, seed=3, impurity="entropy")
    digests = []
    for native in (True, False):
        monkeypatch.setattr(engine.ForestTrainer, "_native_split_ex", lambda self, d, v=native: v and
                            engine.NATIVE_SPLIT and d.type == "cuda")
        m = est.fit(df)
        digests.append(forest_digest(m._forest))
    assert digests[0] == digests[1]


@pytest.mark.parametrize("model", ["rf", "gbt", "xgb_missing"])
def test_device_split_decode_forests_identical(dev, model, monkeypatch):
    """The partition tables decoded on the device (split.hip split_decode_kernel, partition queued before the
    decisions reach the host) give the forests of the host decode bit for bit: numeric RF / GBT splits and
    XGBoost's missing-right bin sets."""
    import cdnaml
    from cdnaml.models.tree import engine
    from cdnaml.utils.synthetic import forest_digest, regression_shard
    from cdnaml.ml.regression import GBTRegressor, RandomForestRegressor
    from cdnaml.ml.xgboost import XgboostRegressor
    spark = cdnaml.SparkSession.builder.getOrCreate()
    X, y, _ = regression_shard(200_000, 30, 7, 0, 1, dev)
    if model == "xgb_missing":
        X = torch.where(X > 1.2, torch.zeros_like(X), X)     # zeros = missing values
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
    est = {"rf": RandomForestRegressor(numTrees=16, maxDepth=6, maxBins=32, seed=3),
           "gbt": GBTRegressor(maxIter=4, maxDepth=5, seed=1),
           "xgb_missing": XgboostRegressor(n_estimators=4, max_depth=6, missing=0.0, random_state=2)}[model]
    digests = []
    for flag in (True, False):
        monkeypatch.setattr(engine, "DEVICE_DECODE", flag)
        digests.append(forest_digest(est.fit(df)._forest))
    assert digests[0] == digests[1]


@pytest.mark.parametrize("flow", ["dt_reg", "rf_reg", "rf_binary", "rf_reg_deep", "rf_binary_deep"])
def test_device_decode_categorical_forests_identical(dev, flow, monkeypatch):
    """Categorical winners decoded on the device (split_decode with split_scan_ex's category bitmasks, partition
    queued before the decisions reach the host) give the host decode's forests bit for bit: regression trees /
    forests with StringIndexer'd categoricals (ML 06) and a binary classifier on the same features, also deeper
    than 8 levels (node-id partition from the device tables)."""
    import cdnaml
    import pandas as pd
    from cdnaml.models.tree import engine
    from cdnaml.utils.synthetic import forest_digest
    from cdnaml.ml.feature import StringIndexer, VectorAssembler
    from cdnaml.ml.classification import RandomForestClassifier
    from cdnaml.ml.regression import DecisionTreeRegressor, RandomForestRegressor
    spark = cdnaml.SparkSession.builder.getOrCreate()
    rng = np.random.default_rng(5)
    n = 60_000
    pdf = pd.DataFrame({"hood": [f"h{i}" for i in rng.integers(0, 37, n)],
                        "room": rng.choice(["entire", "private", "shared", "hotel"], n),
                        "beds": rng.integers(1, 6, n).astype(float), "lat": rng.normal(size=n)})
    hood_num = pdf.hood.str[1:].astype(int)
    price = 40 * pdf.beds + 15 * (hood_num % 5) + 60 * (pdf.room == "entire") + 10 * pdf.lat + rng.normal(size=n) * 5
    pdf["label"] = (price > np.median(price)).astype(float) if flow.startswith("rf_binary") else price
    sdf = spark.createDataFrame(pdf)
    sdf = StringIndexer(inputCols=["hood", "room"], outputCols=["hoodIdx", "roomIdx"]).fit(sdf).transform(sdf)
    df = VectorAssembler(inputCols=["hoodIdx", "roomIdx", "beds", "lat"], outputCol="features").transform(sdf)
    est = {"dt_reg": DecisionTreeRegressor(maxDepth=6, maxBins=40),
           "rf_reg": RandomForestRegressor(numTrees=8, maxDepth=6, maxBins=40, seed=2),
           "rf_binary": RandomForestClassifier(numTrees=8, maxDepth=6, maxBins=40, seed=2),
           # deeper than 8: the node-id levels decode on the device too (node-id partition behind K6)
           "rf_reg_deep": RandomForestRegressor(numTrees=4, maxDepth=11, maxBins=40, seed=2),
           "rf_binary_deep": RandomForestClassifier(numTrees=4, maxDepth=11, maxBins=40, seed=2)}[flow]
    decodes = {"n": 0}
    orig = K.split_decode

    def counted(*a, **k):
        decodes["n"] += int(k.get("catm") is not None)
        return orig(*a, **k)
    monkeypatch.setattr(K, "split_decode", counted)
    digests = []
    for flag in (True, False):
        monkeypatch.setattr(engine, "DEVICE_DECODE", flag)
        digests.append(forest_digest(est.fit(df)._forest))
    assert decodes["n"] > 0  # the categorical device decode ran
    assert digests[0] == digests[1]
