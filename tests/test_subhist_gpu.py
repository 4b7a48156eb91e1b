"""K5s / K6s: feature-subset level histograms with on-the-fly items (subhist.hip) and the compact split scan
(split.hip) vs exact references: the int64 sums against a host index_add over the same items, the split
decisions against the full-feature split kernel on the expanded histogram, and whole forests against the
full-feature + subtraction path (the same forest bit for bit)."""
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


def _level(n, d, B, T, nodes_per_tree, m, seed, dev):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g)
    thr = torch.sort(torch.randn(d, B - 1, generator=g), dim=1).values
    nthr = torch.full((d,), B - 1, dtype=torch.int32)
    bins, rm = K.binize(X.to(dev), thr.to(dev), nthr.to(dev), want_rm=True)
    rng = np.random.default_rng(seed)
    w = np.minimum(rng.poisson(1.0, size=(T, n)), 255)
    loc = rng.integers(0, nodes_per_tree, size=(T, n))
    loc[rng.random((T, n)) < 0.1] = 0xFF                       # rows already in a leaf
    codes = ((w << 8) | np.where(w == 0, 0xFF, loc)).astype(np.int16)
    A = T * nodes_per_tree
    slot_tree = np.repeat(np.arange(T), nodes_per_tree)
    tfirst = np.arange(T) * nodes_per_tree
    feats = np.sort(np.stack([rng.choice(d, m, replace=False) for _ in range(A)]), 1).astype(np.int32)
    v1 = torch.from_numpy(rng.standard_t(3, size=n).astype(np.float32) * 50)
    qs1 = K._packed_scale(v1)
    return bins, rm, torch.from_numpy(codes), v1, qs1, tfirst, slot_tree, feats, int(w.max())


@pytest.mark.parametrize("n,d,B,T,npt,m", [(50_003, 100, 40, 6, 4, 34), (20_000, 100, 40, 3, 16, 34),
                                            (30_000, 64, 32, 5, 2, 10), (40_000, 120, 64, 2, 8, 70),
                                            (10_000, 40, 256, 4, 2, 13)])
def test_sub_hist_exact(dev, n, d, B, T, npt, m):
    bins, rm, codes, v1, qs1, tfirst, slot_tree, feats, wmax = _level(n, d, B, T, npt, m, n + m, dev)
    ref = K.sub_hist(codes, v1, qs1, bins.cpu(), None, tfirst, slot_tree, feats, B, wmax)
    out = K.sub_hist(codes.to(dev), v1.to(dev), qs1, bins, rm, tfirst, slot_tree, feats, B, wmax).cpu()
    assert ref.abs().sum() > 0
    assert torch.equal(out, ref)
    # slot ranges (the multi-rank overlap chunks) compose to the same sums
    S = len(slot_tree)
    part = torch.zeros_like(out).to(dev)
    for s0, s1 in ((0, S // 3), (S // 3, S)):
        K.sub_hist(codes.to(dev), v1.to(dev), qs1, bins, rm, tfirst, slot_tree, feats, B, wmax, s0, s1,
                   out=part[s0:s1])
    assert torch.equal(part.cpu(), ref)


def test_sub_hist_fp64_semantics(dev):
    """Against an fp64 numpy histogram of the same (row, weight, label) items: the count is exact and the
    weighted label sum is the fp64 sum up to the label's 24-bit quantisation."""
    n, d, B, T, npt, m = 30_000, 50, 40, 4, 2, 17
    bins, rm, codes, v1, qs1, tfirst, slot_tree, feats, wmax = _level(n, d, B, T, npt, m, 7, dev)
    out = K.sub_hist(codes.to(dev), v1.to(dev), qs1, bins, rm, tfirst, slot_tree, feats, B, wmax).cpu().double()
    c = codes.numpy().astype(np.int32) & 0xFFFF
    loc, w = c & 0xFF, c >> 8
    flat = bins.cpu().permute(1, 0, 2).reshape(n, -1).numpy()
    y = v1.numpy().astype(np.float64)
    cnt = np.zeros((len(slot_tree), m, B))
    s = np.zeros((len(slot_tree), m, B))
    for t in range(T):
        ok = (loc[t] != 0xFF) & (w[t] > 0)
        rows = np.nonzero(ok)[0]
        sl = tfirst[t] + loc[t, rows]
        for k in range(m):
            f = feats[sl, k]
            np.add.at(cnt, (sl, k, flat[rows, f]), w[t, rows])
            np.add.at(s, (sl, k, flat[rows, f]), w[t, rows] * y[rows])
    np.testing.assert_array_equal(out[..., 0].numpy(), cnt)
    np.testing.assert_allclose(out[..., 1].numpy() / qs1, s, rtol=0, atol=cnt.max() * 1.0 / qs1)


def test_split_scan_sub_equals_full_split(dev):
    n, d, B, T, npt, m = 60_000, 100, 40, 5, 4, 34
    bins, rm, codes, v1, qs1, tfirst, slot_tree, feats, wmax = _level(n, d, B, T, npt, m, 11, dev)
    Hc = K.sub_hist(codes.to(dev), v1.to(dev), qs1, bins, rm, tfirst, slot_tree, feats, B, wmax)
    nthr = torch.full((d,), B - 1, dtype=torch.int32, device=dev)
    nthr[::7] = 20                                               # fewer legal thresholds on some features
    so, tot = K.split_scan_sub(Hc, feats, nthr, qs1, 1.0)
    H = K.sub_hist_expand(Hc, feats, d, qs1)
    A = len(slot_tree)
    words = np.zeros((A, (d + 31) // 32), dtype=np.uint32)
    for a_ in range(A):
        for f in feats[a_]:
            words[a_, f >> 5] |= np.uint32(1) << np.uint32(f & 31)
    # the full kernel's node totals come from the first feature with the largest weight: the first sampled one
    so_f, tot_f = K.split_scan(H, nthr, torch.from_numpy(words.view(np.int32)).to(dev), 0, 1.0)
    assert torch.equal(so.cpu(), so_f.cpu())
    assert torch.equal(tot.cpu(), tot_f.cpu())


@pytest.mark.parametrize("strategy", ["onethird", "sqrt"])
def test_forest_identical_subset_vs_full_feature_path(dev, strategy, monkeypatch):
    """The whole forest through subset histograms equals the full-feature + sibling-subtraction forest."""
    import cdnaml
    from cdnaml.models.regression import RandomForestRegressor
    from cdnaml.models.tree import engine
    from cdnaml.utils.synthetic import forest_digest, regression_shard
    spark = cdnaml.SparkSession.builder.getOrCreate()
    X, y, _ = regression_shard(300_000, 60, 3, 0, 1, dev)
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
    digests = []
    for flag in (False, True):
        monkeypatch.setattr(engine, "SUB_HIST", flag)
        rf = RandomForestRegressor(numTrees=12, maxDepth=6, maxBins=40, seed=5, featureSubsetStrategy=strategy)
        model = rf.fit(df)
        digests.append((model.totalNumNodes, forest_digest(model._forest)))
    assert digests[0] == digests[1]
