"""Transform of a forest's own training tensor from the fit's uint8 bins (forest.FitBins, K.tree_predict_heap_binned).

For a threshold v of the binning, x <= v  <=>  t_bin(x) <= v (t_b = the b-th threshold, +inf for the last bin and
NaN), so the heap walk over the bins' upper edges takes the fp32 walk's branches: the predictions are identical
bit for bit.  CPU: the dequantised walk against the raw walk and the node-path predictor, with values lying exactly
on thresholds, +-inf and NaN.  GPU: the HIP kernel against the fp32 heap kernel, and ``transform`` of the fit's
frame served from the bins only while the tensor is the fit's, unmodified and alive."""
import gc

import numpy as np
import pytest
import torch

from cdnaml.ops import kernels as K


def _fit(spark, X, y, **kw):
    from cdnaml.models.regression import RandomForestRegressor
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
    est = RandomForestRegressor(numTrees=kw.pop("T", 7), maxDepth=kw.pop("depth", 5), maxBins=kw.pop("B", 24),
                                seed=3, minInstancesPerNode=2, **kw)
    return df, est.fit(df)


def _data(n, d, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g)
    X[:, 1] = torch.randint(0, 6, (n,), generator=g).float() * 0.5   # few distinct values: midpoints hit data
    y = (X[:, 0] * 2 - X[:, 1] + torch.sin(X[:, 2]) + 0.1 * torch.randn(n, generator=g)).double()
    return X, y


def _heap(model, dev):
    f = model._forest
    f.settle()
    h = f.heap_arrays(dev, "value")
    tw, = K.upload(dev, np.asarray(model._tree_w, np.float64))
    return h[0], h[1], tw


def test_binned_walk_equals_raw_cpu(spark):
    if spark.device.type != "cpu":
        pytest.skip("host walk")
    from cdnaml.models.tree.binning import make_binned
    n, d = 3000, 13
    X, y = _data(n, d)
    df, m = _fit(spark, X, y)
    heap, D, tw = _heap(m, X.device)
    # the fit's binning, rebuilt (same sample / thresholds: the seed and shapes are the fit's)
    data = make_binned(spark, X, {}, 24, 3, 0, n)
    f = m._forest
    for g in range(len(f.feat)):  # every split threshold is a threshold of this binning (fp32)
        if f.feat[g] >= 0:
            assert np.float32(f.thr[g]) == np.float32(data.thresholds[f.feat[g], f.bin[g]])
    up = torch.from_numpy(K.bin_upper_edges(data.thresholds, data.nthr, 24))
    raw = K.heap_predict_host(X, heap, D, tw)
    nodes, roots, vals, masks = f.device_arrays(X.device)
    ref = K.tree_predict(X, nodes, roots, tw, vals, masks, 1)[:, 0]
    assert torch.equal(raw, ref)
    binned = K.tree_predict_heap_binned(data.bins, up, d, heap, D, tw)[:, 0]
    assert torch.equal(binned, raw)
    # edge values through the same binning: on a threshold, +-inf, NaN, between and beyond the thresholds
    Z = X[:400].clone()
    thr32 = data.thresholds.astype(np.float32)
    for i in range(0, 400, 4):
        f_ = i % d
        k = int(data.nthr[f_])
        Z[i, f_] = float(thr32[f_, i % max(k, 1)]) if k else 0.0
    Z[1, 0], Z[2, 2], Z[3, 0] = float("inf"), float("-inf"), float("nan")
    Z[5, 2] = float("nan")
    zb = K.binize(Z, torch.from_numpy(thr32), torch.from_numpy(data.nthr.astype(np.int32)))
    zb = zb[0] if isinstance(zb, tuple) else zb
    np.testing.assert_array_equal(K.tree_predict_heap_binned(zb, up, d, heap, D, tw)[:, 0].numpy(),
                                  K.heap_predict_host(Z, heap, D, tw).numpy())


def test_fit_bins_lifecycle():
    """FitBins (host tensors): matches only the fit's unmodified, live tensor; one take per fit, exactly one of
    several threads gets the bins; released with the source; never pickled with its forest."""
    import pickle
    import threading
    from cdnaml.models.tree.forest import FitBins, Forest
    X = torch.randn(100, 13)
    bins = torch.zeros((2, 100, 8), dtype=torch.uint8)
    thr = np.sort(np.random.default_rng(0).standard_normal((13, 7)), 1)
    fb = FitBins(X, bins, thr, np.full(13, 7, np.int32), 13, 8)
    assert fb.thr_up.shape == (13, 8) and torch.isinf(fb.thr_up[:, 7]).all()
    assert fb.matches(X) and fb.matches(X.view(100, 13)) and not fb.matches(X.clone())
    got = []
    ths = [threading.Thread(target=lambda: got.append(fb.take(X))) for _ in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert sum(g is not None for g in got) == 1 and fb.bins is None and fb.hits == 1
    assert fb.take(X) is None
    # an in-place write of the source ends the match
    Y = torch.randn(50, 13)
    fy = FitBins(Y, bins, thr, np.full(13, 7, np.int32), 13, 8)
    Y.add_(0.0)
    assert not fy.matches(Y) and fy.take(Y) is None
    # released when the source dies
    Z = torch.randn(20, 13)
    fz = FitBins(Z, bins, thr, np.full(13, 7, np.int32), 13, 8)
    del Z
    gc.collect()
    assert fz.bins is None
    # a forest carrying one pickles without it
    f = Forest(1)
    f._fit_bins = fy
    g = pickle.loads(pickle.dumps(f))
    assert g._fit_bins is None and f._fit_bins is fy


@pytest.mark.gpu
def test_binned_kernel_equals_fp32_kernel(gpu_device):
    import cdnaml
    spark = cdnaml.SparkSession.builder.getOrCreate()
    for n, d, depth, T in ((70001, 100, 5, 20), (4099, 13, 4, 9), (64, 9, 6, 3)):
        X, y = _data(n, d, seed=d)
        Xd, yd = X.to(gpu_device), y.to(gpu_device)
        df, m = _fit(spark, Xd, yd, T=T, depth=depth, B=40)
        fb = m._forest._fit_bins
        assert fb is not None and fb.matches(Xd)
        heap, D, tw = _heap(m, gpu_device)
        for dt in (torch.float64, torch.float32):
            a = K.tree_predict_heap(Xd, heap, D, tw, torch.zeros(8, dtype=torch.int32, device=gpu_device), 0.25,
                                    dtype=dt)
            b = K.tree_predict_heap_binned(fb.bins, fb.thr_up, d, heap, D, tw, 0.25, dtype=dt)
            assert a is not None and b is not None
            assert torch.equal(a, b), (n, d, dt)
        # the host twin of the binned walk agrees too
        a64 = K.tree_predict_heap(Xd, heap, D, tw, torch.zeros(8, dtype=torch.int32, device=gpu_device), 0.25)
        hb = K.tree_predict_heap_binned(fb.bins.cpu(), fb.thr_up.cpu(), d, heap.cpu(), D, tw.cpu(), 0.25)
        assert torch.equal(hb, a64.cpu())


@pytest.mark.gpu
def test_transform_of_fit_frame_uses_bins(gpu_device):
    import cdnaml
    from cdnaml.models.inference import predictor_for
    from cdnaml.models.tree import forest as FM
    spark = cdnaml.SparkSession.builder.getOrCreate()
    X, y = _data(50000, 100, seed=11)
    Xd, yd = X.to(gpu_device), y.to(gpu_device)
    df, m = _fit(spark, Xd, yd, T=20, depth=5, B=40)
    p = predictor_for(m, "value", [m._base])
    fb = m._forest._fit_bins
    assert fb is not None and fb.matches(Xd)
    got = frame_pred(m, df)
    assert p.binned == 1, "transform of the fit's frame did not read the bins"
    assert fb.bins is None  # one transform per fit: released after it
    # the same rows in another tensor, and the fit's frame again after the release: the fp32 path, same values
    df2 = spark.createDataFrameFromLocalTensors({"features": Xd.clone(), "label": yd})
    assert torch.equal(frame_pred(m, df2), got) and torch.equal(frame_pred(m, df), got) and p.binned == 1
    # with the reuse off at fit time: no bins kept, same predictions
    old = FM.REUSE_FIT_BINS
    try:
        FM.REUSE_FIT_BINS = False
        _, m_off = _fit(spark, Xd, yd, T=20, depth=5, B=40)
    finally:
        FM.REUSE_FIT_BINS = old
    assert m_off._forest._fit_bins is None
    assert torch.equal(frame_pred(m_off, df), got)
    # an in-place write after the fit (version bump) ends the match: the fp32 path on the new values
    Xe = Xd.clone()
    dfe, me = _fit(spark, Xe, yd, T=20, depth=5, B=40)
    Xe[0, 0] += 1.0
    assert not me._forest._fit_bins.matches(Xe)
    pe = predictor_for(me, "value", [me._base])
    after = frame_pred(me, dfe)
    assert pe.binned == 0
    ref = frame_pred(me, spark.createDataFrameFromLocalTensors({"features": Xe.clone(), "label": yd}))
    assert torch.equal(after, ref)
    # the bins are released with the source tensor
    X2, y2 = _data(3000, 100, seed=12)
    X2d = X2.to(gpu_device)
    df3, m3 = _fit(spark, X2d, y2.to(gpu_device), T=4, depth=3, B=40)
    fb = m3._forest._fit_bins
    assert fb is not None and fb.bins is not None
    m3._forest.settle()   # the deferred last level's closure holds the trainer (and its frame) until it runs
    del df3, X2d
    gc.collect()
    assert fb.bins is None and not fb.matches(torch.zeros(1, device=gpu_device))


def frame_pred(model, frame):
    parts = model.transform(frame)._plan.execute()
    return torch.cat([b.columns["prediction"].values for b in parts])


@pytest.mark.gpu
def test_fused_sample_same_thresholds(gpu_device, monkeypatch):
    """The one-rank quantile sample gathered on the device (K.sample_gather: NaN-padded to a fixed capacity, no
    host count) gives the exact sample's thresholds and bins; a capacity overflow falls back to the exact sample."""
    import cdnaml
    from cdnaml.models.tree import binning as BN
    spark = cdnaml.SparkSession.builder.getOrCreate()
    g = torch.Generator().manual_seed(4)
    X = torch.randn(300000, 24, generator=g)
    X[:, 3] = torch.randint(0, 5000, (300000,), generator=g).float()
    Xd = X.to(gpu_device)
    outs = {}
    for mode in ("fused", "exact", "overflow"):
        monkeypatch.setattr(BN, "SAMPLE_FUSED", mode != "exact")
        if mode == "overflow":
            real = K.sample_gather

            def fake(*a, **k):
                samp, _ = real(*a, **k)
                return samp, (lambda: False)
            monkeypatch.setattr(K, "sample_gather", fake)
        data = BN._make_binned(spark, Xd, {}, 40, 7, 0, 300000)
        outs[mode] = (data.thresholds.copy(), data.nthr.copy(), data.bins.cpu())
    for mode in ("fused", "overflow"):
        np.testing.assert_array_equal(outs[mode][0], outs["exact"][0])
        np.testing.assert_array_equal(outs[mode][1], outs["exact"][1])
        assert torch.equal(outs[mode][2], outs["exact"][2])
