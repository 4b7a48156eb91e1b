"""CPU reference paths of the kernel library + property tests.

The HIP kernels are checked against these same references on the GPU in
tests/test_kernels_gpu.py; here the references themselves are pinned against
brute-force numpy loops, and the framework-level invariants are property-tested.
"""
import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from cdnaml.ops import kernels as K
from cdnaml.ops import philox


def test_philox_known_answer():
    # Philox4x32-10 known-answer vector (Random123 kat_vectors: counter 0, key 0)
    c = philox.philox4x32_10(np.uint32(0), np.uint32(0), np.uint32(0), np.uint32(0), 0, 0)
    assert [int(x) for x in c] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]


def test_uniform_offsets_are_consistent():
    a = philox.uniform(1000, seed=7)
    b = philox.uniform(300, seed=7, offset=700)
    np.testing.assert_array_equal(a[700:], b)
    assert ((a >= 0) & (a < 1)).all()
    assert abs(a.mean() - 0.5) < 0.05
    t = K.uniform(1000, 7)
    np.testing.assert_array_equal(t.numpy(), a)


def test_normal32_is_keyed_by_global_element():
    """Box-Muller normals from Philox quads: any chunking of the element range gives the same values (the
    inference bench generates its 1e9 rows chunk by chunk), and the moments are those of N(0, 1)."""
    a = philox.normal32(200003, seed=5, offset=0, stream=0x10)
    for off, m in ((0, 7), (1, 10), (3, 4097), (1000, 99003), (200000, 3)):
        np.testing.assert_array_equal(philox.normal32(m, 5, off, 0x10), a[off:off + m])
    assert a.dtype == np.float32
    assert abs(a.mean()) < 0.01 and abs(a.std() - 1.0) < 0.01
    assert abs((np.abs(a) < 1.0).mean() - 0.6827) < 0.005
    t = K.normal32_(torch.empty(100, 3), 5, 6, 0x10)
    np.testing.assert_array_equal(t.reshape(-1).numpy(), a[6:306])


def test_poisson_weights_mean():
    w = K.poisson_weights(4, 20000, seed=3, offset=0, rate=1.0)
    assert w.shape == (4, 20000) and w.dtype == torch.uint8
    m = w.float().mean(1)
    assert torch.all((m - 1.0).abs() < 0.03)
    assert 0.35 < float((w == 0).float().mean()) < 0.39  # e^-1


def _bins(n=500, d=11, B=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g)
    q = torch.linspace(0.05, 0.95, B - 1)
    thr = torch.quantile(X, q, dim=0).T.contiguous()
    nthr = torch.full((d,), B - 1, dtype=torch.int32)
    return X, thr, nthr, K.binize(X, thr, nthr)


def test_binize_matches_searchsorted():
    X, thr, nthr, bins = _bins()
    bm = K.bins_to_matrix(bins, X.shape[1])
    for f in range(X.shape[1]):
        ref = torch.searchsorted(thr[f], X[:, f].contiguous(), right=False)
        assert torch.equal(bm[:, f].long(), ref)


@pytest.mark.parametrize("d", [100, 84, 7])
def test_bins_seg10_layout(d):
    """seg10 rows (the six-items-per-wave histogram's layout, binize rm_layout="s10"): 128 bytes per row, byte
    12 s + p holds feature 10 s + p, the two bytes after each 10-feature chunk and the last 8 bytes are zero."""
    X, thr, nthr, bins = _bins(n=257, d=d, B=40)
    s10 = K.bins_seg10(bins, d)
    assert s10.shape == (257, 16, 8) and s10.dtype == torch.uint8
    flat = s10.reshape(257, 128).long()
    bm = K.bins_to_matrix(bins, d).long()
    used = torch.zeros(128, dtype=torch.bool)
    for f in range(d):
        pos = 12 * (f // 10) + f % 10
        assert torch.equal(flat[:, pos], bm[:, f])
        used[pos] = True
    assert not flat[:, ~used].any()
    with pytest.raises(ValueError):
        K.bins_seg10(torch.zeros((13, 4, 8), dtype=torch.uint8), 101)


def test_hist_moments_bruteforce():
    X, thr, nthr, bins = _bins(n=300, d=5, B=8)
    n, d, B = 300, 5, 8
    T, A = 2, 4
    g = torch.Generator().manual_seed(1)
    node = torch.randint(0, 2, (T, n), generator=g, dtype=torch.int32) + torch.tensor([[0], [2]], dtype=torch.int32)
    build = torch.tensor([0, -1, 1, 2], dtype=torch.int32)
    slot_tree = np.array([0, 1, 1])
    w = K.poisson_weights(T, n, 1, 0, 1.0)
    y = torch.randn(n, generator=g)
    out = K.hist_moments(bins, d, node, w, None, y, build, slot_tree, None, B)
    bm = K.bins_to_matrix(bins, d)
    ref = np.zeros((3, d, B, 2))
    for t in range(T):
        for r in range(n):
            s = int(build[node[t, r]])
            if s < 0:
                continue
            for f in range(d):
                ref[s, f, int(bm[r, f]), 0] += float(w[t, r])
                ref[s, f, int(bm[r, f]), 1] += float(w[t, r]) * float(y[r])
    np.testing.assert_allclose(out.numpy(), ref, rtol=1e-10, atol=1e-10)


def test_fixed_point_scale_bounds():
    v = torch.tensor([1e3, -5.0])
    s = K._fixed_scale(v, 10 ** 8, 255)
    assert 1e8 * 255 * 1e3 * s < 2 ** 62
    assert s >= 2 ** 10
    assert K._fixed_scale(torch.zeros(3), 10, 1) == 1.0
    with pytest.raises(ValueError):
        K._fixed_scale(torch.tensor([float("nan")]), 10, 1)


def test_reg_metrics_and_score_hist():
    g = torch.Generator().manual_seed(0)
    y = torch.randn(1000, generator=g, dtype=torch.float64)
    p = y + 0.1 * torch.randn(1000, generator=g, dtype=torch.float64)
    s = K.reg_metrics(y, p)
    e = (y - p)
    np.testing.assert_allclose(float(s[0]), 1000)
    np.testing.assert_allclose(float(s[1]), float((e * e).sum()), rtol=1e-10)
    lab = (y > 0).double()
    h = K.score_hist(p, lab, -4.0, 4.0, 64)
    assert float(h.sum()) == 1000


def test_kmeans_step_reference():
    g = torch.Generator().manual_seed(0)
    X = torch.randn(200, 3, generator=g)
    C = X[:4].clone()
    assign, sums, counts, cost = K.kmeans_step(X, C)
    d2 = ((X[:, None, :] - C[None]) ** 2).sum(-1)
    assert torch.equal(assign.long(), d2.argmin(1))
    np.testing.assert_allclose(float(cost), float(d2.min(1).values.sum()), rtol=1e-5)
    assert int(counts.sum()) == 200


def test_gram_reference():
    g = torch.Generator().manual_seed(0)
    X = torch.randn(100, 6, generator=g)
    y = torch.randn(100, generator=g)
    G = K.gram(X, y)
    A = torch.cat([X.double(), torch.ones(100, 1, dtype=torch.float64), y.double()[:, None]], 1)
    np.testing.assert_allclose(G.numpy(), (A.T @ A).numpy(), rtol=1e-9, atol=1e-9)


# ----------------------------------------------------------- property tests
@settings(max_examples=25, deadline=None)
@given(n=st.integers(1, 3000), parts=st.integers(1, 9), seed=st.integers(0, 2 ** 31 - 1))
def test_uniform_partition_invariant(n, parts, seed):
    """Counter-based RNG: generating in any number of pieces gives the same stream."""
    whole = philox.uniform(n, seed)
    cuts = np.linspace(0, n, parts + 1).astype(int)
    pieces = np.concatenate([philox.uniform(b - a, seed, offset=a) for a, b in zip(cuts[:-1], cuts[1:])])
    np.testing.assert_array_equal(whole, pieces)


@settings(max_examples=15, deadline=None)
@given(n=st.integers(20, 400), split=st.integers(1, 19), seed=st.integers(0, 1000))
def test_histogram_is_additive(n, split, seed):
    """Histograms of row shards sum to the histogram of the whole (the all-reduce contract)."""
    X, thr, nthr, bins = _bins(n=n, d=3, B=8, seed=seed)
    cut = max(1, n * split // 20)
    node = torch.zeros((1, n), dtype=torch.int32)
    build = torch.tensor([0], dtype=torch.int32)
    y = torch.randn(n, generator=torch.Generator().manual_seed(seed))
    whole = K.hist_moments(bins, 3, node, None, None, y, build, np.array([0]), None, 8)
    a = K.hist_moments(bins[:, :cut].contiguous(), 3, node[:, :cut].contiguous(), None, None, y[:cut], build,
                       np.array([0]), None, 8)
    b = K.hist_moments(bins[:, cut:].contiguous(), 3, node[:, cut:].contiguous(), None, None, y[cut:], build,
                       np.array([0]), None, 8)
    np.testing.assert_allclose((a + b).numpy(), whole.numpy(), rtol=1e-9, atol=1e-9)


@settings(max_examples=10, deadline=None)
@given(seed=st.integers(0, 10000), frac=st.floats(0.1, 0.9))
def test_random_split_partition_count_invariant(seed, frac):
    import cdnaml
    spark = cdnaml.SparkSession.builder.getOrCreate()
    a = spark.range(0, 2000, numPartitions=1).randomSplit([frac, 1 - frac], seed=seed)[0]
    b = spark.range(0, 2000, numPartitions=6).randomSplit([frac, 1 - frac], seed=seed)[0]
    assert set(a.toPandas().id) == set(b.toPandas().id)


def test_find_thresholds_vectorised_matches_host():
    """The batched (device) split-candidate finder is bit-identical to the per-feature host finder
    (Spark findSplits semantics: midpoints of distinct values, or of quantile cut points)."""
    import torch
    from cdnaml.models.tree.engine import find_thresholds, find_thresholds_t
    rng = np.random.default_rng(0)
    for trial in range(20):
        s, d = int(rng.integers(1, 2000)), int(rng.integers(1, 10))
        X = rng.normal(size=(s, d))
        for f in range(d):
            kind = rng.integers(0, 5)
            if kind == 1:
                X[:, f] = rng.integers(0, rng.integers(1, 60), s)
            elif kind == 2:
                X[rng.random(s) < 0.3, f] = np.nan
            elif kind == 3:
                X[:, f] = np.round(X[:, f], 1)
            elif kind == 4:
                X[:, f] = 1.0
        cat = {f: int(np.nanmax(np.abs(X[:, f])) + 1) for f in range(d)
               if rng.random() < 0.15 and not np.isnan(X[:, f]).any()}
        for B in (2, 5, 40, 256):
            a = find_thresholds(X, d, B, cat)
            b = find_thresholds_t(torch.from_numpy(X), B, cat)
            np.testing.assert_array_equal(a[1], b[1])
            np.testing.assert_array_equal(a[0], b[0])


def test_col_moments_reference_semantics():
    """K20 reference path: Spark describe semantics (nulls skipped, NaN propagates to mean/max)."""
    X = torch.tensor([[1.0, 2.0], [3.0, float("nan")], [5.0, 4.0]], dtype=torch.float64)
    v = torch.tensor([[True, True], [True, True], [False, True]])
    m = K.col_moments(X, v)
    assert m[0, 0] == 2 and m[0, 1] == 2.0 and m[0, 2] == 2.0 and m[0, 3] == 1.0 and m[0, 4] == 3.0
    assert m[1, 0] == 3 and torch.isnan(m[1, 1]) and m[1, 3] == 2.0 and torch.isnan(m[1, 4])
    parts = torch.stack([K.col_moments(X[:2]), K.col_moments(X[2:])])
    merged = K._merge_moments(parts)
    full = K.col_moments(X)
    assert torch.allclose(merged[0], full[0])



def test_native_seg_plan_matches_numpy():
    """csrc/kernels/plan.hip (host code of the native library): the record histograms' chunk and work list equal
    the numpy _fill_chunk + _seg_work bit for bit (same chunk, same items in the same interleaved order)."""
    import numpy as np
    from cdnaml.ops import kernels as K
    rng = np.random.default_rng(5)
    cases = 0
    for S in (1, 2, 3, 40, 80, 160, 700):
        for scale in (1e3, 3e5, 2e6, 2e7):
            lens = rng.integers(0, int(scale), S)
            lens[rng.random(S) < 0.1] = 0
            segs = np.stack([np.concatenate([[0], np.cumsum(lens)[:-1]]), lens, np.arange(S)], 1)
            for chunk in (8192, 40960, 786000):
                for B, ncu in ((40, 256), (40, 0), (128, 256)):
                    for inter in (False, True):
                        c_ref = K._fill_chunk(segs, chunk, B, ncu)
                        w_ref = K._seg_work(segs, c_ref, inter)
                        c, w = K._seg_plan(segs, chunk, B, ncu, inter)
                        assert c == c_ref, (S, scale, chunk, B, ncu)
                        np.testing.assert_array_equal(w, w_ref)
                        cases += 1
    assert cases > 500
