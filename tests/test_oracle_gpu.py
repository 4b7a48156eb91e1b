"""fp64 oracles for the split rules the headline and the L07 lab use:

* regression with per-node feature subsets (featureSubsetStrategy "auto" = onethird: 34 of 100 features, the
  headline's masked split path): every internal node's split must be the fp64 variance-gain optimum over THAT
  node's sampled features only (the subsets re-derived from the engine's (seed, tree, heap key) hash);
* classification, Gini and entropy, 3 classes (class-count kernels) and 2 classes (the packed record path,
  engine.MSEG_CLS): every internal node's split must be the fp64 impurity-gain optimum of its rows' exact class
  counts.

Rows are routed through each fitted tree by their bins, so each level is checked against sums recomputed from
scratch in fp64 (not from the engine's histograms).  Zero tolerance violations at every level."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sessions():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import cdnaml
    from cdnaml.ops import _lib
    _lib.lib()
    return cdnaml.SparkSession.builder.getOrCreate()


def _impurity(c, kind):
    W = c.sum(-1, keepdim=True)
    p = c / W.clamp(min=1e-300)
    if kind == "gini":
        return 1.0 - (p * p).sum(-1)
    return -(torch.where(p > 0, p * torch.log2(p.clamp(min=1e-300)), torch.zeros_like(p))).sum(-1)


def _check_levels(f, trainer, bm, w, stats, kind, d, B, depth_max, masks):
    """Route rows; at every level, each internal node's (feature, bin) must attain the fp64 best gain over its
    allowed features.  stats: [n, K] per-row fp64 statistics (regression: (1, y); classes: one-hot)."""
    dev = bm.device
    n = bm.shape[0]
    feat = torch.tensor(f.feat, device=dev)
    binv = torch.tensor(f.bin, device=dev)
    left = torch.tensor(f.left, device=dev)
    right = torch.tensor(f.right, device=dev)
    Kc = stats.shape[1]
    checked = 0
    for t in range(len(f.roots)):
        wt = w[t].double()
        node = torch.full((n,), f.roots[t], dtype=torch.int64, device=dev)
        key = {f.roots[t]: 1}
        for depth in range(depth_max):
            nodes = torch.unique(node)
            inner = nodes[feat[nodes] >= 0]
            if inner.numel() == 0:
                break
            S_ = inner.numel()
            slot = torch.full((len(f.feat),), -1, dtype=torch.int64, device=dev)
            slot[inner] = torch.arange(S_, device=dev)
            rs = slot[node]
            rows = torch.nonzero((rs >= 0) & (wt > 0)).flatten()
            H = torch.zeros((S_ * d * B, Kc), dtype=torch.float64, device=dev)
            idx = (rs[rows, None] * d + torch.arange(d, device=dev)[None, :]) * B + bm[rows]
            H.index_add_(0, idx.reshape(-1), (wt[rows, None] * stats[rows]).repeat_interleave(d, 0))
            H = H.view(S_, d, B, Kc)
            cl = H.cumsum(2)[:, :, :-1]
            tot = H.sum(2, keepdim=True)
            cr = tot - cl
            if kind == "variance":
                WL, SL, WR, SR = cl[..., 0], cl[..., 1], cr[..., 0], cr[..., 1]
                W, S = tot[..., 0], tot[..., 1]
                ok = (WL > 0) & (WR > 0)
                gain = (SL * SL / WL.clamp(min=1) + SR * SR / WR.clamp(min=1) - S * S / W) / W
            else:
                WL, WR, W = cl.sum(-1), cr.sum(-1), tot.sum(-1)
                ok = (WL > 0) & (WR > 0)
                gain = _impurity(tot, kind) - WL / W * _impurity(cl, kind) - WR / W * _impurity(cr, kind)
            gain = torch.where(ok, gain, torch.full_like(gain, -float("inf")))
            if masks:
                keys = np.array([key[int(a)] for a in inner.tolist()], dtype=np.uint64)
                words = trainer._feature_masks(np.full(S_, t, dtype=np.uint64), keys)
                fm = torch.from_numpy(((words[:, np.arange(d) >> 5] >> (np.arange(d) & 31).astype(np.uint32)) & 1)
                                      .astype(bool)).to(dev)
                gain = torch.where(fm[:, :, None], gain, torch.full_like(gain, -float("inf")))
                assert bool(fm[torch.arange(S_, device=dev), feat[inner]].all()), (t, depth)  # split on a sampled feature
            best = gain.reshape(S_, -1).max(1).values
            ours = gain[torch.arange(S_, device=dev), feat[inner], binv[inner]]
            bad = ours < best - 1e-9 * best.abs()
            assert not bool(bad.any()), (t, depth, inner[bad][:4].tolist(), ours[bad][:4].tolist(),
                                         best[bad][:4].tolist())
            checked += S_
            for a in inner.tolist():
                key[f.left[a]] = 2 * key[a]
                key[f.right[a]] = 2 * key[a] + 1
            go_left = bm.gather(1, feat[node].clamp(min=0)[:, None])[:, 0] <= binv[node]
            node = torch.where(feat[node] >= 0, torch.where(go_left, left[node], right[node]), node)
    return checked


def test_masked_regression_splits_are_fp64_optimal(sessions):
    """Headline split rule: RandomForestRegressor featureSubsetStrategy auto -> 34 of 100 features per node."""
    from cdnaml.models.tree.engine import ForestTrainer, TreeParams, make_binned
    from cdnaml.ops import kernels as K
    dev = torch.device("cuda:0")
    n, d, T, B, D = 1_000_000, 100, 20, 40, 5
    g = torch.Generator(device=dev).manual_seed(5)
    X = torch.randn((n, d), generator=g, device=dev)
    y = (X[:, 0] * 2 - X[:, 1] + torch.sin(3 * X[:, 2]) + 0.4 * X[:, 3] * X[:, 4] +
         0.3 * torch.randn(n, generator=g, device=dev))
    data = make_binned(sessions, X, {}, B, 1, 0, n)
    w = K.poisson_weights(T, n, 9, 0, 1.0, device=dev)
    p = TreeParams(max_depth=D, max_bins=B, feature_subset=34, seed=42)
    tr = ForestTrainer(sessions, data, p)
    f = tr.train(T, {"v0": None, "v1": y.float()}, w)
    bm = K.bins_to_matrix(data.bins, d)
    yq = y.float().double()
    checked = _check_levels(f, tr, bm, w, torch.stack([torch.ones_like(yq), yq], 1), "variance", d, B, D, True)
    assert checked >= T * 15


@pytest.mark.parametrize("C,kind", [(3, "gini"), (3, "entropy"), (2, "gini"), (2, "entropy")])
def test_classification_splits_are_fp64_optimal(sessions, C, kind):
    from cdnaml.models.tree.engine import ForestTrainer, TreeParams, make_binned
    from cdnaml.ops import kernels as K
    dev = torch.device("cuda:0")
    n, d, T, B, D = 1_000_000, 100, 6, 40, 5
    g = torch.Generator(device=dev).manual_seed(C * 7 + len(kind))
    X = torch.randn((n, d), generator=g, device=dev)
    z = X[:, 0] * 1.5 - X[:, 1] + torch.sin(2 * X[:, 2]) + 0.5 * torch.randn(n, generator=g, device=dev)
    y = torch.bucketize(z, torch.tensor([-0.5, 0.7], device=dev)) if C == 3 else (z > 0.1).long()
    data = make_binned(sessions, X, {}, B, 1, 0, n)
    w = K.poisson_weights(T, n, 13, 0, 1.0, device=dev)
    p = TreeParams(max_depth=D, max_bins=B, impurity=kind, num_classes=C, feature_subset=None, seed=7)
    tr = ForestTrainer(sessions, data, p)
    f = tr.train(T, {"label": y.int()}, w)
    bm = K.bins_to_matrix(data.bins, d)
    onehot = torch.nn.functional.one_hot(y, C).double()
    checked = _check_levels(f, tr, bm, w, onehot, kind, d, B, D, False)
    assert checked >= T * 10
