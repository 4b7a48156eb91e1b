"""Binary classification forests on the packed record / segment path (engine.MSEG_CLS): with y in {0, 1} at scale 1
the packed sums are (W, W1), turned into class counts in int64, so the forests must equal the class-histogram
kernels' forests bit for bit -- at depth <= 8 (codes, root kernels, records) and deeper (node ids from level 8),
for Gini and entropy (the L07 lab: maxDepth {2, 5, 10} x numTrees {10, 20, 100}, maxBins 40)."""
import pytest
import torch

from cdnaml.ops import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spark():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _lib.lib()
    import cdnaml
    return cdnaml.SparkSession.builder.getOrCreate()


@pytest.mark.parametrize("n,d,T,depth,imp", [(200_000, 100, 20, 5, "gini"), (150_000, 100, 10, 10, "gini"),
                                             (100_003, 24, 6, 6, "entropy"), (80_000, 100, 3, 11, "entropy")])
def test_packed_classification_forest_equals_class_histograms(spark, n, d, T, depth, imp):
    from cdnaml.models.classification import RandomForestClassifier
    from cdnaml.models.tree import engine
    from cdnaml.ops import kernels as K
    from cdnaml.utils.synthetic import forest_digest
    g = torch.Generator(device="cuda").manual_seed(n + depth)
    X = torch.randn((n, d), generator=g, device="cuda")
    y = ((X[:, 0] * 2 - X[:, 1] + torch.sin(3 * X[:, 2]) + 0.5 * torch.randn(n, generator=g, device="cuda")) > 0)
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": y.double()})
    est = RandomForestClassifier(numTrees=T, maxDepth=depth, maxBins=40, seed=7, impurity=imp)
    out, calls = [], []
    orig_c, orig_s = K.seg_hist_codes, K.seg_hist
    for flag in (False, True):
        cnt = {"n": 0}

        def counted_c(*a, **k):
            cnt["n"] += 1
            return orig_c(*a, **k)

        def counted_s(*a, **k):
            cnt["n"] += 1
            return orig_s(*a, **k)
        engine.MSEG_CLS = flag
        K.seg_hist_codes, K.seg_hist = counted_c, counted_s
        try:
            out.append(forest_digest(est.fit(df)._forest))
        finally:
            engine.MSEG_CLS = True
            K.seg_hist_codes, K.seg_hist = orig_c, orig_s
        calls.append(cnt["n"])
    # the packed path ran (root levels from the codes at d = 100, record histograms below / at other widths)
    assert calls[0] == 0 and calls[1] >= 1, calls
    assert out[0] == out[1]
