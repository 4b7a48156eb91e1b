"""Numerics of every native HIP kernel vs its plain-PyTorch CPU reference."""
import math

import pandas as pd
import numpy as np
import pytest
import torch

from cdnaml.ops import _lib, kernels as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _lib.lib()  # must load: no silent fallback on a GPU box
    return torch.device("cuda:0")


@pytest.mark.parametrize("n,d", [(1000, 5), (4097, 30), (20000, 100), (333, 200)])
def test_gram_f32(dev, n, d):
    g = torch.Generator().manual_seed(n + d)
    X = torch.randn(n, d, generator=g) * 3 + 1
    y = torch.randn(n, generator=g)
    sh = X[:64].mean(0)
    ref = K.gram(X, y, sh, 0.25)
    out = K.gram(X.to(dev), y.to(dev), sh.to(dev), 0.25).cpu()
    assert torch.allclose(out, ref, rtol=1e-5, atol=1e-3 * n ** 0.5)


def test_gram_asymmetric_identity(dev):
    # A = I-check with asymmetric data: catches row/col swaps in the C layout
    n, d = 64, 40
    X = torch.arange(n * d, dtype=torch.float32).reshape(n, d) % 7 - (torch.arange(d) % 5)[None, :]
    ref = K.gram(X)
    out = K.gram(X.to(dev)).cpu()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("n,d,shifted,ldx", [(5000, 100, False, None), (100, 7, False, None),
                                             (70001, 128, True, None), (200003, 64, True, None), (3, 4, True, None),
                                             (9000, 100, True, 101), (131, 156, False, None)])
def test_gram_bf16(dev, n, d, shifted, ldx):
    # d % 4 == 0 with aligned rows takes the streaming kernel; ldx=101 / d=7 the tiled fallback
    g = torch.Generator().manual_seed(7 + n)
    X = torch.randn(n, ldx or d, generator=g) * 2 + 0.5
    y = torch.randn(n, generator=g) + 3
    sh = X[:64, :d].mean(0) if shifted else None
    ys = 2.5 if shifted else 0.0
    Xd = X.to(dev)[:, :d]
    X = X[:, :d]
    ref = K.gram(X.contiguous(), y, sh, ys, bf16=True)
    out = K.gram(Xd, y.to(dev), None if sh is None else sh.to(dev), ys, bf16=True).cpu()
    assert torch.allclose(out, ref, rtol=1e-4, atol=1e-2 * max(1.0, n / 20000))


def test_uniform_bit_identical(dev):
    a = K.uniform(100000, 42, 12345, 3)
    b = K.uniform(100000, 42, 12345, 3, device=dev).cpu()
    assert torch.equal(a, b)


@pytest.mark.parametrize("n,offset,shift", [(100000, 0, 0), (100003, 5, 0), (4097, 2, 1), (3, 7, 0), (1, 0, 3)])
def test_normal32_matches_host_oracle(dev, n, offset, shift):
    """float4 stores (aligned output, offset % 4 == 0) and per-element stores (unaligned offset or output
    pointer) against the host oracle (the same fp32 uniforms, float64 log/sin/cos): only the kernel's hardware
    log/sin/cos differ."""
    ref = torch.from_numpy(__import__("cdnaml.ops.philox", fromlist=["normal32"]).normal32(n, 9, offset, 0x10))
    buf = torch.full((n + shift + 1,), 7.0, device=dev)
    out = K.normal32_(buf[shift:shift + n], 9, offset, 0x10).cpu()
    assert torch.allclose(out, ref, rtol=2e-4, atol=2e-4)
    tail = buf.cpu()
    assert tail[n + shift].item() == 7.0 and (shift == 0 or tail[shift - 1].item() == 7.0)


@pytest.mark.parametrize("rate,n,offset", [(1.0, 50000, 1000), (0.63, 50000, 1000), (2.5, 50000, 1000),
                                           (1.0, 50003, 1001), (7.5, 4099, 6)])
def test_poisson_matches(dev, rate, n, offset):
    """Integer-threshold draws (8 unrolled compares, CDF loop past 7, exact tail) with dword stores of interior
    quads (aligned) or byte stores (unaligned offsets / row lengths) equal the host Philox reference."""
    a = K.poisson_weights(4, n, 7, offset, rate)
    b = K.poisson_weights(4, n, 7, offset, rate, device=dev).cpu()
    assert (a != b).sum().item() <= 2  # libm exp() may differ in the last ulp


def _thresholds(X, maxb):
    d = X.shape[1]
    thr = torch.zeros(d, maxb - 1)
    nthr = torch.zeros(d, dtype=torch.int32)
    for f in range(d):
        q = torch.quantile(X[:2000, f], torch.linspace(0, 1, maxb + 1)[1:-1]).unique()
        thr[f, : len(q)] = q
        nthr[f] = len(q)
    return thr, nthr


def test_binize(dev):
    g = torch.Generator().manual_seed(1)
    X = torch.randn(3000, 21, generator=g)
    X[:, 3] = torch.randint(0, 9, (3000,), generator=g).float()
    thr, nthr = _thresholds(X, 40)
    nthr[3] = -1
    X[5, 2] = float("nan")
    ref = K.binize(X, thr, nthr)
    out = K.binize(X.to(dev), thr.to(dev), nthr.to(dev)).cpu()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("lut", [256, 64, 0])
def test_binize_lut_columns(dev, lut, monkeypatch):
    """binize v6 (uniform-grid LUT + a short walk of the value's cell) equals the host count #{t < x} exactly on
    columns the grid fits badly: heavy tails (lognormal, Cauchy: the wave falls back to the binary search),
    a constant column (one threshold), two thresholds, a narrow far-from-zero column, +-inf / NaN values and
    values equal to thresholds; the row-major seg10 copy too."""
    monkeypatch.setattr(K, "BINIZE_LUT", lut)
    g = torch.Generator().manual_seed(9)
    n, d = 20003, 24
    X = torch.randn(n, d, generator=g)
    X[:, 1] = torch.exp(3 * X[:, 1])                          # lognormal
    X[:, 2] = torch.tan(3.1 * (torch.rand(n, generator=g) - 0.5))  # Cauchy-like
    X[:, 3] = 7.0                                             # constant
    X[:, 4] = torch.randint(0, 3, (n,), generator=g).float()  # three values
    X[:, 5] = 37.8 + 0.02 * X[:, 5]                           # latitude-like
    X[:, 6] = torch.round(X[:, 6] * 4) / 4                    # ties with the thresholds
    X[::97, 7] = float("inf")
    X[::89, 7] = float("-inf")
    X[::13, 8] = float("nan")
    thr, nthr = _thresholds(X.nan_to_num(0.0, posinf=0.0, neginf=0.0), 40)
    X[:50, 6] = thr[6, 0]                                     # exactly on a threshold
    ref = K.binize(X, thr, nthr)
    out, rm = K.binize(X.to(dev), thr.to(dev), nthr.to(dev), want_rm=True, rm_layout="s10")
    assert torch.equal(out.cpu(), ref)
    assert torch.equal(rm.cpu(), K.bins_seg10(ref.to(dev), d).cpu())


@pytest.mark.parametrize("max_bins,s,f32", [(40, 10000, False), (256, 16384, False), (2, 3000, False),
                                            (32, 777, False), (40, 10000, True), (40, 12288, True),
                                            (40, 12289, True), (256, 5000, True)])
def test_quantile_thresholds_kernel(dev, max_bins, s, f32):
    """K3 quantile kernel == the host findSplits reference (NaNs, +-inf, few-distinct and categorical columns).
    f32: every column exactly fp32 (the engine's samples), so s <= 12288 takes the radix-sorted path for all."""
    from cdnaml.models.tree.engine import find_thresholds, find_thresholds_t
    g = torch.Generator().manual_seed(max_bins + s)
    samp = torch.randn(s, 37, generator=g, dtype=torch.float64)
    if f32:
        samp = samp.float().double()
    samp[:, 3] = torch.randint(0, 6, (s,), generator=g).double()       # categorical
    samp[:, 4] = torch.round(samp[:, 4] * 3)                             # few distinct values
    samp[::5, 7] = float("nan")
    samp[::11, 8] = float("inf")
    samp[::13, 8] = -float("inf")
    samp[:, 9] = float("nan")                                            # empty column
    samp[: s // 2, 10] = 2.5                                             # heavy tie at one value
    cats = {3: 6}
    q = K.quantile_thresholds(samp.to(dev), max_bins)
    assert q is not None
    thr_d, nthr_d = find_thresholds_t(samp.to(dev), max_bins, cats)
    thr_h, nthr_h = find_thresholds(samp.numpy(), 37, max_bins, cats)
    assert np.array_equal(nthr_d, nthr_h)
    assert np.array_equal(thr_d, thr_h, equal_nan=True)
    # the device-threshold path: the kernel's own fp32 copy is the fp64 thresholds rounded (the binning's input)
    qd = K.quantile_thresholds_dev(samp.to(dev), max_bins)
    if qd is not None:
        t32, n32, pend = qd
        t64, ints = pend.get()
        assert t32.dtype == torch.float32 and np.array_equal(n32.cpu().numpy(), ints[0])
        t32h = t32.cpu().numpy()
        for f in range(37):  # the thresholds in use (nthr of them; the host path redoes the others)
            k = int(ints[0][f])
            assert np.array_equal(t32h[f, :k], t64[f, :k].astype(np.float32)), f


@pytest.mark.parametrize("d", [21, 100])
def test_binize_row_major_copy(dev, d):
    """The binning kernel's row-major copy equals the standalone transpose (padding words zeroed)."""
    g = torch.Generator().manual_seed(2)
    X = torch.randn(4099, d, generator=g)
    thr, nthr = _thresholds(X, 40)
    bins, rm = K.binize(X.to(dev), thr.to(dev), nthr.to(dev), want_rm=True)
    assert rm is not None
    ref = K.bins_row_major(bins)
    assert rm.shape == ref.shape
    assert torch.equal(rm.cpu(), ref.cpu())
    assert torch.equal(bins.cpu(), K.binize(X, thr, nthr))


def _tree_state(n, T, A, seed):
    g = torch.Generator().manual_seed(seed)
    node = torch.randint(-1, A, (T, n), generator=g, dtype=torch.int32)
    build = torch.randint(-1, 3, (A,), generator=g, dtype=torch.int32)
    # slots must be tree-major: remap per tree (ids are tree-major: A/T ids per tree)
    per = A // T
    slot_tree = []
    s = 0
    for i in range(A):
        if build[i] >= 0:
            build[i] = s
            slot_tree.append(i // per)
            s += 1
    for t in range(T):
        lo, hi = t * per, (t + 1) * per
        m = node[t] >= 0
        node[t][m] = lo + (node[t][m] % per)
    return node, build, np.array(slot_tree, np.int32)


def _set_hist_version(monkeypatch, ver):
    """ver: 4 = the v4 integer kernel with the lane-per-row mapping (hist4_kernel); 46 = the fast rotated
    kernel (hist4f_kernel)."""
    monkeypatch.setattr(K, "HIST_MAP", 5 if ver == 46 else 2)


@pytest.mark.parametrize("B", [40, 256])
@pytest.mark.parametrize("ver", [4, 46])
def test_hist_moments(dev, B, ver, monkeypatch):
    n, d, T, A = 20000, 19, 3, 12
    g = torch.Generator().manual_seed(B)
    X = torch.randn(n, d, generator=g)
    thr, nthr = _thresholds(X, B)
    bins = K.binize(X, thr, nthr)
    node, build, slot_tree = _tree_state(n, T, A, 3)
    S = len(slot_tree)
    w = K.poisson_weights(T, n, 5, 0, 1.0)
    y = torch.randn(n, generator=g)
    mw = (d + 31) // 32
    fm = torch.randint(0, 2 ** 31 - 1, (S, mw), generator=g, dtype=torch.int64).to(torch.int32)
    id_tree = np.arange(A) // (A // T)
    _set_hist_version(monkeypatch, ver)
    ref = K.hist_moments(bins, d, node, w, None, y, build, slot_tree, fm, B)
    out = K.hist_moments(bins.to(dev), d, node.to(dev), w.to(dev), None, y.to(dev), build.to(dev), slot_tree,
                         fm.to(dev), B, lds_budget=8 * 1024, id_tree=id_tree).cpu()
    assert torch.allclose(out, ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("ver", [4, 46])
def test_hist_classes(dev, ver, monkeypatch):
    n, d, T, A, C, B = 10000, 10, 2, 8, 3, 32
    g = torch.Generator().manual_seed(11)
    X = torch.randn(n, d, generator=g)
    thr, nthr = _thresholds(X, B)
    bins = K.binize(X, thr, nthr)
    node, build, slot_tree = _tree_state(n, T, A, 4)
    w = K.poisson_weights(T, n, 5, 0, 1.0)
    lab = torch.randint(0, C, (n,), generator=g, dtype=torch.int32)
    ref = K.hist_classes(bins, d, node, w, lab, C, build, slot_tree, None, B)
    id_tree = np.arange(A) // (A // T)
    _set_hist_version(monkeypatch, ver)
    out = K.hist_classes(bins.to(dev), d, node.to(dev), w.to(dev), lab.to(dev), C, build.to(dev), slot_tree, None,
                         B, id_tree=id_tree).cpu()
    assert torch.allclose(out, ref)


@pytest.mark.parametrize("ver", [4])
def test_hist_moments_v0(dev, ver, monkeypatch):
    """Moments with a real-valued v0 plane (XGBoost hessians) and no bootstrap weights."""
    n, d, T, A, B = 30000, 13, 2, 6, 64
    g = torch.Generator().manual_seed(5)
    X = torch.randn(n, d, generator=g)
    thr, nthr = _thresholds(X, B)
    bins = K.binize(X, thr, nthr)
    node, build, slot_tree = _tree_state(n, T, A, 6)
    v0 = torch.rand(n, generator=g) * 0.25
    v1 = torch.randn(n, generator=g) * 100.0
    _set_hist_version(monkeypatch, ver)
    ref = K.hist_moments(bins, d, node, None, v0, v1, build, slot_tree, None, B)
    out = K.hist_moments(bins.to(dev), d, node.to(dev), None, v0.to(dev), v1.to(dev), build.to(dev), slot_tree,
                         None, B, id_tree=np.arange(A) // (A // T)).cpu()
    assert torch.allclose(out, ref, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("ver", [4, 46])
def test_hist_v4_deterministic(dev, ver, monkeypatch):
    """Integer histograms are bit-identical across launches with different chunkings."""
    n, d, T, A, B = 50000, 16, 2, 4, 32
    g = torch.Generator().manual_seed(8)
    X = torch.randn(n, d, generator=g)
    thr, nthr = _thresholds(X, B)
    bins = K.binize(X, thr, nthr).to(dev)
    node, build, slot_tree = _tree_state(n, T, A, 2)
    y = torch.randn(n, generator=g).to(dev)
    _set_hist_version(monkeypatch, ver)
    it = np.arange(A) // (A // T)
    a = K.hist_moments(bins, d, node.to(dev), None, None, y, build.to(dev), slot_tree, None, B, id_tree=it)
    b = K.hist_moments(bins, d, node.to(dev), None, None, y, build.to(dev), slot_tree, None, B, lds_budget=4096,
                       id_tree=it)
    assert torch.equal(a, b)


def test_partition(dev):
    n, d, T, A = 5000, 12, 2, 6
    g = torch.Generator().manual_seed(2)
    X = torch.randn(n, d, generator=g)
    X[:, 4] = torch.randint(0, 20, (n,), generator=g).float()
    thr, nthr = _thresholds(X, 32)
    nthr[4] = -1
    bins = K.binize(X, thr, nthr)
    node, _, _ = _tree_state(n, T, A, 9)
    sf = torch.tensor([0, 4, -1, 7, 4, 11], dtype=torch.int32)
    sb = torch.tensor([10, 0, 0, 3, 0, 20], dtype=torch.int32)
    co = torch.tensor([-1, 0, -1, -1, 1, -1], dtype=torch.int32)
    cm = torch.randint(0, 2 ** 31 - 1, (16,), generator=g, dtype=torch.int64).to(torch.int32)
    child = torch.arange(12, dtype=torch.int32) - 2
    a = node.clone()
    K.partition(bins, a, sf, sb, co, cm, child)
    b = node.to(dev)
    K.partition(bins.to(dev), b, sf.to(dev), sb.to(dev), co.to(dev), cm.to(dev), child.to(dev))
    assert torch.equal(a, b.cpu())


def _random_forest_arrays(T, depth, d, K_, seed):
    g = torch.Generator().manual_seed(seed)
    nodes, values, roots = [], [], []
    masks = torch.randint(0, 2 ** 31 - 1, (4 * 8,), generator=g, dtype=torch.int64).to(torch.int32)
    for t in range(T):
        roots.append(len(nodes))
        base = len(nodes)
        nint = 2 ** depth - 1
        for i in range(nint):
            l, r = base + 2 * i + 1, base + 2 * i + 2
            if i % 5 == 4:
                nodes.append([-(int(torch.randint(0, d, (1,), generator=g)) + 2), i % 4, l, r])
            else:
                thr = float(torch.randn(1, generator=g))
                nodes.append([int(torch.randint(0, d, (1,), generator=g)),
                              int(torch.tensor([thr], dtype=torch.float32).view(torch.int32)), l, r])
        for i in range(2 ** depth):
            nodes.append([-1, len(values), 0, 0])
            values.extend(torch.randn(K_, generator=g).tolist())
    return (torch.tensor(nodes, dtype=torch.int32), torch.tensor(roots, dtype=torch.int32),
            torch.tensor(values, dtype=torch.float64), masks)


@pytest.mark.parametrize("K_", [1, 3])
def test_tree_predict(dev, K_):
    n, d, T = 3000, 17, 7
    g = torch.Generator().manual_seed(K_)
    X = torch.randn(n, d, generator=g)
    X[:, 3] = torch.randint(0, 40, (n,), generator=g).float()
    nodes, roots, values, masks = _random_forest_arrays(T, 4, d, K_, 5)
    # categorical nodes use feature 3 only
    cat = nodes[:, 0] < -1
    nodes[cat, 0] = -(3 + 2)
    tw = torch.rand(T, generator=g, dtype=torch.float64)
    base = torch.randn(K_, generator=g, dtype=torch.float64)
    ref = K.tree_predict(X, nodes, roots, tw, values, masks, K_, base)
    out = K.tree_predict(X.to(dev), nodes.to(dev), roots.to(dev), tw.to(dev), values.to(dev), masks.to(dev), K_,
                         base.to(dev)).cpu()
    # fp64 leaves / weights / sums in one fixed tree order on both devices: bit-identical
    assert out.dtype == torch.float64 and torch.equal(out, ref)


def test_reg_metrics(dev):
    g = torch.Generator().manual_seed(3)
    y = torch.randn(100001, generator=g, dtype=torch.float64)
    p = y + 0.1 * torch.randn(100001, generator=g, dtype=torch.float64)
    ref = K.reg_metrics(y, p)
    out = K.reg_metrics(y.to(dev), p.to(dev)).cpu()
    assert torch.allclose(out, ref, rtol=1e-10)


def test_kmeans_step(dev):
    g = torch.Generator().manual_seed(3)
    X = torch.randn(10000, 4, generator=g)
    C = torch.randn(5, 4, generator=g)
    a1, s1, c1, cost1 = K.kmeans_step(X, C)
    a2, s2, c2, cost2 = K.kmeans_step(X.to(dev), C.to(dev))
    assert torch.equal(a1, a2.cpu())
    assert torch.allclose(s1, s2.cpu(), rtol=1e-5, atol=1e-3)
    assert torch.allclose(c1, c2.cpu())


def test_logistic_grad(dev):
    g = torch.Generator().manual_seed(3)
    X = torch.randn(20000, 37, generator=g)
    y = (torch.rand(20000, generator=g) > 0.5).double()
    w = torch.randn(37, generator=g, dtype=torch.float64) * 0.1
    g1, l1 = K.logistic_grad(X, y, w, 0.3)
    g2, l2 = K.logistic_grad(X.to(dev), y.to(dev), w.to(dev), 0.3)
    assert torch.allclose(g1, g2.cpu(), rtol=1e-4, atol=1e-3)
    assert abs(float(l1) - float(l2)) < 1e-3 * abs(float(l1))


def test_score_hist(dev):
    g = torch.Generator().manual_seed(3)
    s = torch.rand(50000, generator=g, dtype=torch.float64)
    lab = (torch.rand(50000, generator=g) > 0.3).double()
    assert torch.equal(K.score_hist(s, lab, 0.0, 1.0, 1000), K.score_hist(s.to(dev), lab.to(dev), 0.0, 1.0, 1000).cpu())


def _codes_state(n, T, per, seed):
    """Random row records: T trees with `per` active nodes each (tree-major ids)."""
    g = torch.Generator().manual_seed(seed)
    w = K.poisson_weights(T, n, seed, 0, 1.0)
    codes = K.codes_init(w, T, n, "cpu")
    loc = torch.randint(0, per, (T, n), generator=g, dtype=torch.int32)
    done = torch.rand((T, n), generator=g) < 0.1
    c = codes.to(torch.int32) & 0xFFFF
    loc = torch.where(done | ((c & 0xFF) == 0xFF), torch.full_like(loc, 0xFF), loc)
    codes = ((c & 0xFF00) | loc).to(torch.int16).contiguous()
    tfirst = torch.arange(T, dtype=torch.int32) * per
    A = T * per
    build = torch.randint(-1, 2, (A,), generator=g, dtype=torch.int32)
    slot_tree, s = [], 0
    for i in range(A):
        if build[i] >= 0:
            build[i] = s
            slot_tree.append(i // per)
            s += 1
    id_tree = np.arange(A) // per
    return codes, tfirst, build, np.array(slot_tree, dtype=np.int32), id_tree


@pytest.mark.parametrize("kind", ["moments", "moments_v0", "classes", "masked", "packed", "packed_masked",
                                  "packed_wmax", "packed_nc", "packed_nc_masked", "packed_big", "packed_big_masked",
                                  "packed_q", "packed_q_masked", "packed_q_wmax"])
def test_hist_codes(dev, kind, monkeypatch):
    # packed_q_*: wave-compacted kernel (hist5q) forced; packed_nc_*: lane-per-row packed kernel
    # (hist5p) only; packed / packed_big: automatic choice (*_big: 128 KB plane -> 1024-thread blocks,
    # where the compacted kernel is chosen)
    n, d, T, per, B, C = 30000, 21, 18, 5, 40, 3
    g = torch.Generator().manual_seed(7)
    X = torch.randn(n, d, generator=g)
    thr, nthr = _thresholds(X, B)
    bins = K.binize(X, thr, nthr)
    codes, tfirst, build, slot_tree, id_tree = _codes_state(n, T, per, 3)
    S = len(slot_tree)
    y = torch.randn(n, generator=g) * 10
    h = torch.rand(n, generator=g)
    lab = torch.randint(0, C, (n,), generator=g, dtype=torch.int32)
    fm = None
    monkeypatch.setattr(K, "HIST5_PACKED", kind.startswith("packed"))
    monkeypatch.setattr(K, "HIST5_COMPACT", 0 if kind.startswith("packed_nc") else
                        2 if kind.startswith("packed_q") else 1)
    if kind.endswith("masked"):
        fm = torch.randint(0, 2 ** 31 - 1, (S, (d + 31) // 32), generator=g, dtype=torch.int64).to(torch.int32)
    mode = 1 if kind == "classes" else 0
    v0 = h if kind == "moments_v0" else None
    ref = K.hist_codes(mode, bins, d, codes, tfirst, v0, y, lab, C, build, slot_tree, id_tree, fm, B)
    wmax = int(((codes.to(torch.int32) & 0xFFFF) >> 8).max()) if kind.endswith("wmax") else 255
    out = K.hist_codes(mode, bins.to(dev), d, codes.to(dev), tfirst, None if v0 is None else v0.to(dev), y.to(dev),
                       lab.to(dev), C, build.to(dev), slot_tree, id_tree, None if fm is None else fm.to(dev), B,
                       lds_budget=(128 if "big" in kind else 16) * 1024, wmax=wmax).cpu()
    assert torch.allclose(out, ref, rtol=1e-6, atol=1e-3)


@pytest.mark.parametrize("variant,n,T,d", [("p5", 20000, 6, 12), ("p5", 4000, 3, 130), ("p7", 20001, 6, 12),
                                           ("p7", 70001, 30, 100), ("p7", 20000, 6, 12)])
def test_partition_codes(dev, monkeypatch, variant, n, T, d):
    monkeypatch.setattr(K, "PARTITION7", variant == "p7")
    monkeypatch.setattr(K, "PARTITION7_MIN_T", 1)
    per = 4
    g = torch.Generator().manual_seed(5)
    X = torch.randn(n, d, generator=g)
    X[:, 3] = torch.randint(0, 20, (n,), generator=g).float()
    thr, nthr = _thresholds(X, 32)
    nthr[3] = -1
    bins = K.binize(X, thr, nthr)
    codes, tfirst, _, _, _ = _codes_state(n, T, per, 9)
    A = T * per
    sf = torch.randint(-1, d, (A,), generator=g, dtype=torch.int32)
    sb = torch.randint(0, 30, (A,), generator=g, dtype=torch.int32)
    co = torch.where(sf == 3, torch.arange(A, dtype=torch.int32) % 2, torch.full((A,), -1, dtype=torch.int32))
    cm = torch.randint(0, 2 ** 31 - 1, (16,), generator=g, dtype=torch.int64).to(torch.int32)
    # next level: 2 children per node, some finished
    child = torch.arange(2 * A, dtype=torch.int32)
    child[torch.rand(2 * A, generator=g) < 0.2] = -1
    tfirst_next = torch.arange(T, dtype=torch.int32) * (2 * per)
    a = codes.clone()
    K.partition_codes(bins, a, tfirst, tfirst_next, sf, sb, co, cm, child)
    b = codes.to(dev)
    K.partition_codes(bins.to(dev), b, tfirst, tfirst_next, sf, sb, co, cm.to(dev), child)
    assert torch.equal(a, b.cpu())


def _seg_state(n, d, B, nseg, seed, weights):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g)
    thr, nthr = _thresholds(X, B)
    bins = K.binize(X, thr, nthr)
    keep = torch.rand(n, generator=g) < 0.8
    perm = torch.nonzero(keep).flatten().int()
    perm = perm[torch.randperm(perm.numel(), generator=g)]
    m = perm.numel()
    cuts = np.sort(np.random.default_rng(seed).choice(np.arange(1, m), nseg - 1, replace=False))
    starts = np.concatenate([[0], cuts])
    lens = np.diff(np.concatenate([starts, [m]]))
    v1 = torch.randn(m, generator=g) * 5
    v0 = torch.rand(m, generator=g)
    wp = torch.randint(0, 4, (m,), generator=g, dtype=torch.uint8) if weights else None
    return bins, perm, v0, v1, wp, np.stack([starts, lens], 1)


@pytest.mark.parametrize("packed,weights,B,d", [(True, False, 256, 100), (True, True, 40, 21), (True, True, 40, 100), (False, False, 64, 13),
                                                 (False, True, 256, 9)])
@pytest.mark.parametrize("row_major", [False, True, "pad"])
def test_seg_hist(dev, packed, weights, B, d, row_major):
    bins, perm, v0, v1, wp, segs = _seg_state(30000, d, B, 7, 3, weights)
    build = [0, 2, 3, 6]
    sb = np.array([[segs[a, 0], segs[a, 1], i] for i, a in enumerate(build)])
    v0a = None if packed else v0
    ref = K.seg_hist(bins, d, B, perm, v0a, v1, wp, sb, len(build), 3)
    bd = bins.to(dev)
    out = K.seg_hist(bd, d, B, perm.to(dev), None if v0a is None else v0a.to(dev), v1.to(dev),
                     None if wp is None else wp.to(dev), sb, len(build), 3,
                     bins_rm=(K.bins_row_major(bd, pad=True) if row_major == "pad" else
                              bd.permute(1, 0, 2).contiguous() if row_major else None)).cpu()
    assert torch.allclose(out, ref, rtol=1e-6, atol=1e-3)


@pytest.mark.parametrize("with_v0,weights", [(False, False), (True, True)])
def test_seg_partition(dev, with_v0, weights):
    n, d, B = 40000, 12, 32
    bins, perm, v0, v1, wp, segs = _seg_state(n, d, B, 5, 9, weights)
    # segment 1 is a leaf (rows dropped); segment 3 is a categorical-mask split; others ordered splits
    sf = np.array([2, -1, 5, 0, 11], dtype=np.int32)
    sbin = np.array([10, 0, 3, 20, 15], dtype=np.int32)
    co = np.array([-1, -1, -1, 0, -1], dtype=np.int32)
    cm = np.random.default_rng(1).integers(0, 2 ** 31 - 1, 8).astype(np.int32)
    # children: seg0 -> (0, 1), seg2 -> (2, leaf), seg3 -> (3, 4), seg4 -> (leaf, 5)
    child = np.array([0, 1, -1, -1, 2, -1, 3, 4, -1, 5], dtype=np.int32)
    v0a = v0 if with_v0 else None
    ref = K.seg_partition(bins, perm, v0a, v1, wp, segs, sf, sbin, co, cm, child, 6)
    out = K.seg_partition(bins.to(dev), perm.to(dev), None if v0a is None else v0a.to(dev), v1.to(dev),
                          None if wp is None else wp.to(dev), segs, sf, sbin, co, cm, child, 6)
    np.testing.assert_array_equal(ref[4], out[4])
    assert torch.equal(ref[0].int(), out[0].cpu())  # stable: same order as the reference
    assert torch.equal(ref[2], out[2].cpu())
    if with_v0:
        assert torch.equal(ref[1], out[1].cpu())
    if weights:
        assert torch.equal(ref[3], out[3].cpu())


def test_seg_partition_implicit_level0(dev):
    """Multi-tree entry: tree t's root segment is every row, weight-0 rows are dropped (stable)."""
    n, d, B, T = 30000, 12, 32, 5
    bins = _seg_state(n, d, B, 1, 4, False)[0]
    gen = torch.Generator().manual_seed(11)
    v0, v1 = torch.rand(n, generator=gen), torch.randn(n, generator=gen) * 5
    w = torch.from_numpy(np.random.default_rng(5).poisson(1.0, (T, n)).clip(0, 255).astype(np.uint8))
    segs = np.stack([np.arange(T) * n, np.full(T, n)], 1)
    sf = np.array([2, -1, 5, 0, 11], dtype=np.int32)
    sbin = np.array([10, 0, 3, 20, 15], dtype=np.int32)
    co = np.array([-1, -1, -1, 0, -1], dtype=np.int32)
    cm = np.random.default_rng(1).integers(0, 2 ** 31 - 1, 8).astype(np.int32)
    child = np.array([0, 1, -1, -1, 2, -1, 3, 4, -1, 5], dtype=np.int32)
    ref = K.seg_partition(bins, None, v0, v1, w, segs, sf, sbin, co, cm, child, 6)
    out = K.seg_partition(bins.to(dev), None, v0.to(dev), v1.to(dev), w.to(dev), segs, sf, sbin, co, cm, child, 6)
    np.testing.assert_array_equal(ref[4], out[4])
    assert torch.equal(ref[0].int(), out[0].cpu())
    assert torch.equal(ref[1], out[1].cpu()) and torch.equal(ref[2], out[2].cpu())
    assert torch.equal(ref[3], out[3].cpu())
    assert int(ref[3].min()) > 0  # out-of-bag rows dropped


@pytest.mark.parametrize("rank", [None, 0, 1, 2, 3])
@pytest.mark.parametrize("max_loc", [9, 17])
@pytest.mark.parametrize("waves", [2048, 4])
def test_codes_compact(dev, monkeypatch, rank, max_loc, waves):
    """Rows of built nodes gathered into slot segments: same (row, v1, w) multiset per slot as the reference.
    rank None = the atomic (not wave-owned) kernel; else the wave-owned kernel ranking a node's lanes by ballots
    (0) or a DPP prefix scan (1; from one built node up), both stable: exactly the reference order; 2 = the queued
    scatter of packed records (codes_scatter_q_kernel), the same records; 3 = the queued scatter loading one trip
    ahead.  max_loc 17 reaches 16 built nodes per tree (KB = 16); waves 4 gives each wave ~25 trips (the queue's
    carry between trips)."""
    monkeypatch.setattr(K, "COMPACT_W", rank is not None)
    monkeypatch.setattr(K, "COMPACT_WAVES", waves)
    monkeypatch.setattr(K, "SCATTER_QUEUE", rank in (2, 3))
    monkeypatch.setattr(K, "SCATTER_PREFETCH", rank == 3)
    if rank is not None:
        monkeypatch.setattr(K, "SCATTER_RANK", min(rank, 1))
        monkeypatch.setattr(K, "SCATTER_SCAN_MIN_KB", 1)
    T, n = 6, 50000
    rng = np.random.default_rng(2 + max_loc)
    nloc = rng.integers(1, max_loc, T)
    tfirst = torch.from_numpy(np.concatenate([[0], np.cumsum(nloc)[:-1]]).astype(np.int32))
    A = int(nloc.sum())
    loc = rng.integers(0, max_loc, (T, n))
    loc = np.where(loc >= nloc[:, None], 0xFF, loc)
    w = rng.integers(1, 5, (T, n))
    codes = torch.from_numpy(((w << 8) | loc).astype(np.uint16).view(np.int16))
    build = rng.random(A) < 0.6
    slot_of = np.full(A, -1, np.int32)
    slot_of[build] = np.arange(build.sum())
    S = int(build.sum())
    v1 = torch.randn(n)
    ref = K.codes_compact(codes, tfirst, slot_of, S, None, v1)
    out = K.codes_compact(codes.to(dev), tfirst, slot_of, S, None, v1.to(dev))
    np.testing.assert_array_equal(ref[4], out[4])
    for s_, (st, ln) in enumerate(ref[4]):
        key_r = sorted(zip(ref[0][st:st + ln].tolist(), ref[3][st:st + ln].tolist()))
        key_o = sorted(zip(out[0][st:st + ln].cpu().tolist(), out[3][st:st + ln].cpu().tolist()))
        assert key_r == key_o
        rows = out[0][st:st + ln].long().cpu()
        assert torch.equal(out[2][st:st + ln].cpu(), v1[rows])
    if rank is not None:
        assert torch.equal(out[0].cpu(), ref[0]) and torch.equal(out[3].cpu(), ref[3])
        # packed records through the same ranking
        sc = 1024.0
        rec, _, _, _, sg = K.codes_compact(codes.to(dev), tfirst, slot_of, S, None, v1.to(dev), rec_scale=sc)
        rref, _, _, _, _ = K.codes_compact(codes, tfirst, slot_of, S, None, v1, rec_scale=sc)
        np.testing.assert_array_equal(sg, ref[4])
        assert torch.equal(rec.cpu(), rref)


def test_bins_row_major(dev):
    bins = torch.randint(0, 255, (13, 100003, 8), dtype=torch.uint8)
    ref = bins.permute(1, 0, 2).contiguous()
    assert torch.equal(K.bins_row_major(bins.to(dev), pad=False).cpu(), ref)
    padded = K.bins_row_major(bins.to(dev), pad=True).cpu()
    assert padded.shape == (100003, 16, 8)
    assert torch.equal(padded[:, :13], ref) and int(padded[:, 13:].abs().sum()) == 0


def test_mseg_forest_matches_codes_forest(dev, monkeypatch):
    """RandomForest through multi-tree segment mode builds the codes-mode forest."""
    import cdnaml
    from cdnaml.models.tree import engine as E
    from cdnaml.ml.regression import RandomForestRegressor
    spark = cdnaml.SparkSession.builder.getOrCreate()
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn((300000, 24), generator=g, device=dev)
    y = (X[:, 0] * 2 + torch.sin(X[:, 1] * 3) + (X[:, 2] > 0.5).float()).double()
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
    preds = []
    for mseg in (False, True):
        monkeypatch.setattr(E, "USE_MSEG", mseg)
        m = RandomForestRegressor(numTrees=8, maxDepth=6, maxBins=40, seed=7).fit(df)
        preds.append(m.transform(df).select("prediction").toPandas().prediction.values)
    assert np.abs(preds[0] - preds[1]).max() < 1e-3


def test_seg_mode_matches_codes_mode(dev, monkeypatch):
    """One-tree fits (XGBoost rounds, DecisionTree) through the segment kernels give the codes-mode model."""
    import cdnaml
    from cdnaml.models.tree import engine as E
    from cdnaml.ml.feature import VectorAssembler
    from cdnaml.ml.regression import DecisionTreeRegressor
    from cdnaml.ml.xgboost import XgboostRegressor
    spark = cdnaml.SparkSession.builder.getOrCreate()
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn((200000, 20), generator=g, device=dev)
    y = (X[:, 0] * 2 + torch.sin(X[:, 1] * 3) + (X[:, 2] > 0.5).float()).double()
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
    for mk in (lambda: DecisionTreeRegressor(maxDepth=7), lambda: XgboostRegressor(n_estimators=4, max_depth=6)):
        preds = []
        # codes-only, node-segment partition, row records + per-level compaction
        for seg, t1 in ((False, False), (True, False), (False, True)):
            monkeypatch.setattr(E, "USE_SEG", seg)
            monkeypatch.setattr(E, "MSEG_T1", t1)
            preds.append(mk().fit(df).transform(df).select("prediction").toPandas().prediction.values)
        assert np.abs(preds[0] - preds[1]).max() < 1e-3
        assert np.abs(preds[0] - preds[2]).max() < 1e-3


@pytest.mark.parametrize("nonneg,implicit,rank", [(False, False, 12), (True, False, 4), (False, True, 8),
                                                  (True, True, 20)])
def test_als_native_matches_torch_path(dev, monkeypatch, nonneg, implicit, rank):
    """K12 (als.hip accumulate + batched Cholesky/NNLS) against the torch reference half-steps."""
    import cdnaml
    import pandas as pd
    from cdnaml.models import recommendation as R
    spark = cdnaml.SparkSession.builder.getOrCreate()
    rng = np.random.default_rng(3)
    nu, ni, nnz = 300, 200, 6000
    u = rng.integers(0, nu, nnz)
    i = rng.integers(0, ni, nnz)
    Ut, Vt = rng.normal(size=(nu, 3)), rng.normal(size=(ni, 3))
    rt = np.clip((Ut[u] * Vt[i]).sum(1) + 3 + 0.3 * rng.normal(size=nnz), 0.5, 5.0)
    df = spark.createDataFrame(pd.DataFrame({"userId": u, "movieId": i, "rating": rt}))
    preds = []
    for native in (False, True):
        monkeypatch.setattr(R, "ALS_NATIVE", native)
        m = R.ALS(userCol="userId", itemCol="movieId", ratingCol="rating", rank=rank, maxIter=5, regParam=0.1,
                  nonnegative=nonneg, implicitPrefs=implicit, seed=42).fit(df)
        preds.append(np.asarray(m.itemFactors.toPandas().features.tolist(), dtype=np.float64))
    np.testing.assert_allclose(preds[1], preds[0], rtol=1e-4, atol=1e-5)


def test_codes_init_kernel(dev):
    w = torch.randint(0, 7, (5, 10007), dtype=torch.uint8)
    w[2, 5] = 200
    ref, ref_max = K.codes_init_max(w, 5, 10007, "cpu")
    out, mx = K.codes_init_max(w.to(dev), 5, 10007, dev)
    assert torch.equal(ref, out.cpu()) and mx == ref_max == 200


@pytest.mark.parametrize("dtype,d,with_valid", [(torch.float32, 100, False), (torch.float64, 3, True),
                                                (torch.float64, 70, True)])
def test_col_moments(dev, dtype, d, with_valid):
    """K20 one-pass column moments vs the fp64 torch reference (nulls skipped, NaN max/mean)."""
    g = torch.Generator().manual_seed(1)
    n = 200003
    X = (torch.randn(n, d, generator=g, dtype=torch.float64) * 3 + 1).to(dtype)
    X[5, 0] = float("nan") if d == 3 else X[5, 0]
    v = (torch.rand(n, d, generator=g) > 0.1) if with_valid else None
    ref = K.col_moments(X, v)
    out = K.col_moments(X.to(dev), None if v is None else v.to(dev)).cpu()
    assert torch.equal(out[:, 0], ref[:, 0])
    assert torch.allclose(out[:, 1:3], ref[:, 1:3], rtol=1e-9, atol=1e-9, equal_nan=True)
    assert torch.equal(out[:, 3:], ref[:, 3:]) or torch.allclose(out[:, 3:], ref[:, 3:], equal_nan=True)


@pytest.mark.parametrize("W", [2, 8, 37, 1000])
def test_partition_dest(dev, W):
    """K16 stable counting sort == stable argsort of the destination bucket."""
    g = torch.Generator().manual_seed(W)
    dest = torch.randint(0, W, (300001,), generator=g)
    perm, counts = K.partition_dest(dest.to(dev), W)
    assert torch.equal(perm.cpu(), torch.argsort(dest, stable=True))
    assert torch.equal(counts.cpu(), torch.bincount(dest, minlength=W))


def test_heap_predict_matches_node_predict(dev, monkeypatch):
    """K8 heap-layout walk == int4-node walk (categorical splits, NaN features, GBT weighted leaves)."""
    import cdnaml
    from cdnaml.models.tree import forest as F
    from cdnaml.ml.regression import RandomForestRegressor, GBTRegressor
    spark = cdnaml.SparkSession.builder.getOrCreate()
    g = torch.Generator(device=dev).manual_seed(3)
    X = torch.randn((50000, 12), generator=g, device=dev)
    X[:, 4] = torch.randint(0, 9, (50000,), generator=g, device=dev).float()
    y = (X[:, 0] * 2 + torch.sin(X[:, 1] * 3) + (X[:, 4] == 3).float() * 2).double()
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
    Xq = X.clone()
    Xq[::97, 0] = float("nan")
    for est in (RandomForestRegressor(numTrees=7, maxDepth=6, seed=1), GBTRegressor(maxIter=5, maxDepth=4)):
        m = est.fit(df)
        f = m._forest
        tw = m._tree_w if hasattr(m, "_tree_w") and len(m._tree_w) else np.full(len(f.roots), 1.0 / len(f.roots))
        outs = []
        for heap in (True, False):
            monkeypatch.setattr(F, "HEAP_PREDICT", heap)
            outs.append(f.predict(Xq, tw).cpu())
        assert torch.allclose(outs[0], outs[1], rtol=1e-6, atol=1e-5)


def test_compact_records_histogram(dev):
    """Packed item records (row | w | quantised label) give the same segment histograms as perm/v1/w."""
    T, n, d, B = 5, 60000, 21, 40
    rng = np.random.default_rng(8)
    nloc = np.full(T, 2)
    tfirst = torch.from_numpy(np.arange(T, dtype=np.int32) * 2)
    loc = rng.integers(0, 3, (T, n))
    loc = np.where(loc == 2, 0xFF, loc)
    w = rng.integers(0, 6, (T, n))
    loc = np.where(w == 0, 0xFF, loc)
    codes = torch.from_numpy(((w << 8) | loc).astype(np.uint16).view(np.int16)).to(dev)
    slot_of = np.array([0, -1, 1, -1, -1, 2, 3, 4, 5, -1], dtype=np.int32)
    S = 6
    g = torch.Generator().manual_seed(2)
    X = torch.randn(n, d, generator=g)
    thr, nthr = _thresholds(X, B)
    bins = K.binize(X.to(dev), thr.to(dev), nthr.to(dev))
    rm = K.bins_row_major(bins)
    v1 = (torch.randn(n, generator=g) * 3).to(dev)
    sc = K.seg_scales(None, v1, 5, n)
    p0, _, v1p, wp, sg = K.codes_compact(codes, tfirst, slot_of, S, None, v1)
    r1, _, nv, nw, sg1 = K.codes_compact(codes, tfirst, slot_of, S, None, v1, rec_scale=sc[1])
    assert nv is None and r1.dtype == torch.int64
    np.testing.assert_array_equal(sg, sg1)
    assert torch.equal(r1 & 0x7FFFFFFF, p0.long())
    sb = np.concatenate([sg, np.arange(S)[:, None]], 1)
    a = K.seg_hist(bins, d, B, p0, None, v1p, wp, sb, S, 5, sc, bins_rm=rm)
    b = K.seg_hist(bins, d, B, r1, None, None, None, sb, S, 5, sc, bins_rm=rm, rec=True)
    assert torch.equal(a, b)
    # the CPU emulation (gloo ranks) produces the same int64 fixed-point histograms from the same codes
    bins_c, v1_c = bins.cpu(), v1.cpu()
    r_c, _, _, _, sg_c = K.codes_compact(codes.cpu(), tfirst, slot_of, S, None, v1_c, rec_scale=sc[1])
    np.testing.assert_array_equal(sg, sg_c)
    raw_g = K.seg_hist(bins, d, B, r1, None, None, None, sb, S, 5, sc, bins_rm=rm, rec=True, raw=True).cpu()
    raw_c = K.seg_hist(bins_c, d, B, r_c, None, None, None, sb, S, 5, sc, rec=True, raw=True)
    assert raw_g.dtype == raw_c.dtype == torch.int64 and torch.equal(raw_g, raw_c)
    # non-record segment paths too (packed and two-statistic), raw int64
    pc, _, v1pc, wpc, _ = K.codes_compact(codes.cpu(), tfirst, slot_of, S, None, v1_c)
    ga = K.seg_hist(bins, d, B, p0, None, v1p, wp, sb, S, 5, sc, bins_rm=rm, raw=True).cpu()
    ca = K.seg_hist(bins_c, d, B, pc, None, v1pc, wpc, sb, S, 5, sc, raw=True)
    assert torch.equal(ga, ca)
    v0 = (torch.rand(n, generator=g) + 0.1).to(dev)
    sc2 = K.seg_scales(v0, v1, 5, n)
    p2, v0p, v1p2, wp2, _ = K.codes_compact(codes, tfirst, slot_of, S, v0, v1)
    p2c, v0pc, v1p2c, wp2c, _ = K.codes_compact(codes.cpu(), tfirst, slot_of, S, v0.cpu(), v1_c)
    gb = K.seg_hist(bins, d, B, p2, v0p, v1p2, wp2, sb, S, 5, sc2, bins_rm=rm, raw=True).cpu()
    cb = K.seg_hist(bins_c, d, B, p2c, v0pc, v1p2c, wp2c, sb, S, 5, sc2, raw=True)
    assert torch.equal(gb, cb)


def test_native_split_scan_matches_torch(dev, monkeypatch):
    """K6 split kernel == torch split search: RF (feature subsets), DecisionTree, XGBoost (lambda/gamma)."""
    import cdnaml
    from cdnaml.models.tree import engine as E
    from cdnaml.ml.regression import DecisionTreeRegressor, RandomForestRegressor
    from cdnaml.ml.xgboost import XgboostRegressor
    spark = cdnaml.SparkSession.builder.getOrCreate()
    g = torch.Generator(device=dev).manual_seed(5)
    X = torch.randn((100000, 16), generator=g, device=dev)
    y = (X[:, 0] * 2 + torch.sin(X[:, 1] * 3) + (X[:, 2] > 0.5).float()).double()
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
    for mk in (lambda: RandomForestRegressor(numTrees=6, maxDepth=6, seed=3),
               lambda: DecisionTreeRegressor(maxDepth=7, minInstancesPerNode=20),
               lambda: XgboostRegressor(n_estimators=3, max_depth=5, reg_lambda=2.0, gamma=0.1)):
        preds = []
        for native in (False, True):
            monkeypatch.setattr(E, "NATIVE_SPLIT", native)
            preds.append(mk().fit(df).transform(df).select("prediction").toPandas().prediction.values)
        assert np.abs(preds[0] - preds[1]).max() < 1e-4


@pytest.mark.parametrize("A,d,B,kind,missing,masked", [(7, 100, 256, 1, False, False), (33, 37, 256, 1, True, False),
                                                       (5, 100, 200, 0, False, True), (12, 300, 100, 0, False, False),
                                                       (3, 64, 65, 1, True, True), (9, 13, 129, 0, False, False)])
def test_split_scan_wave_bit_identical(dev, A, d, B, kind, missing, masked, monkeypatch):
    """K6 over exact histograms (B > 64): the wave-parallel kernel (a wave per feature, split_scan_wave_kernel)
    returns the serial kernel's bits -- gains, winners (incl. the serial walk's tie order: empty bins make runs of equal gains,
    and with no missing rows every missing-right candidate ties its left twin), left / right sums, node totals."""
    g = torch.Generator().manual_seed(A * d + B)
    cnt = torch.randint(0, 50, (A, d, B), generator=g).double()
    cnt[torch.rand((A, d, B), generator=g) < 0.4] = 0.0  # empty bins: equal-gain runs
    if missing:
        cnt[: A // 2, :, 0] = 0.0  # half the nodes without missing rows: left / right twins tie
    s = torch.randint(-(1 << 20), 1 << 20, (A, d, B), generator=g).double() * cnt.sign() * 2.0 ** -14
    H = torch.stack([cnt, s], -1)
    nthr = torch.randint(B // 2, B + 1, (d,), generator=g).int()
    nthr[d // 3] = -1  # a feature with no legal threshold
    masks = None
    if masked:
        bits = torch.rand((A, d), generator=g) < 0.5
        words = torch.zeros((A, (d + 31) // 32), dtype=torch.int64)
        for f in range(d):
            words[:, f >> 5] |= bits[:, f].long() << (f & 31)
        masks = words.to(torch.int32)
    Hd = H.to(dev)
    outs = []
    for exact in (False, True):
        monkeypatch.setattr(K, "SPLIT_WAVE", True)
        so, tot = K.split_scan(Hd, nthr.to(dev), None if masks is None else masks.to(dev), kind, 1.0, 1.5, 0.0,
                               1.0, missing_bin=missing, exact=exact)
        outs.append((so.cpu(), tot.cpu()))
    assert torch.equal(outs[0][1], outs[1][1])
    a, b = outs[0][0], outs[1][0]
    assert torch.equal(a[:, 1:], b[:, 1:]), (a[:, :3], b[:, :3])
    assert torch.equal(a[:, 0], b[:, 0])


def test_split_scan_wave_same_boosted_forest(dev, monkeypatch):
    """The boosting rounds take the wave-parallel K6 (exact packed histograms) and partition from the feature-major
    byte copy: the forest (and the margins the partitions update) are the serial kernel's / the [G][n] words'."""
    import cdnaml
    from cdnaml.ml.xgboost import XgboostRegressor
    from cdnaml.utils.synthetic import forest_digest
    spark = cdnaml.SparkSession.builder.getOrCreate()
    g = torch.Generator(device=dev).manual_seed(9)
    X = torch.randn((200000, 40), generator=g, device=dev)
    y = (X[:, 0] * 2 + torch.sin(X[:, 1] * 3) + (X[:, 2] > 0.5).float()).double()
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
    digests, preds = [], []
    for wave, fm in ((False, False), (True, False), (True, True)):
        monkeypatch.setattr(K, "SPLIT_WAVE", wave)
        monkeypatch.setattr(K, "PART_FEATURE_MAJOR", fm)  # partition5 from the feature-major byte copy
        m = XgboostRegressor(n_estimators=4, max_depth=8, max_bin=256, learning_rate=0.3).fit(df)
        digests.append(forest_digest(m._forest))
        preds.append(m.transform(df).select("prediction").toPandas().prediction.values)
    assert digests[0] == digests[1] == digests[2]
    assert np.array_equal(preds[0], preds[1]) and np.array_equal(preds[0], preds[2])


@pytest.mark.parametrize("n,p", [(1000003, 0.3), (4097, 0.0), (50000, 1.0)])
def test_compact_mask(dev, n, p):
    """K19 stream compaction == torch.nonzero order."""
    g = torch.Generator().manual_seed(n)
    m = torch.rand(n, generator=g) < p
    assert torch.equal(K.compact_mask(m.to(dev)).cpu(), torch.nonzero(m).flatten())


@pytest.mark.parametrize("missing", [float("nan"), 0.0])
def test_binize_missing_in_kernel(dev, missing):
    """XGBoost missing values (NaN, or == missing) go to bin 0 inside the binning kernel."""
    g = torch.Generator().manual_seed(6)
    X = torch.randn(20000, 13, generator=g)
    X[::7, 2] = float("nan")
    X[::5, 3] = 0.0
    thr, nthr = _thresholds(X.nan_to_num(0.0), 30)
    thr = torch.cat([torch.full((13, 1), -torch.finfo(torch.float32).max), thr], 1)
    nthr = nthr + 1
    ref = K.binize(X, thr, nthr, missing=missing)
    out = K.binize(X.to(dev), thr.to(dev), nthr.to(dev), missing=missing).cpu()
    assert torch.equal(out, ref)
    assert int(out[0, ::7, 2].max()) == 0


@pytest.mark.parametrize("obj", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("weighted", [False, True])
def test_grad_hess_kernel(dev, obj, weighted):
    """K9 gradient/hessian kernel vs the fp32 torch formulas of every supported objective."""
    g0 = torch.Generator().manual_seed(obj)
    n, C = 5003, (4 if obj == 5 else 1)
    F = torch.randn(n, C, generator=g0)
    if obj == 5:
        y = torch.randint(0, C, (n,), generator=g0).float()
    elif obj == 4:
        y = torch.randint(0, 2, (n,), generator=g0).float()
    elif obj == 3:
        y = torch.randint(0, 5, (n,), generator=g0).float()
    else:
        y = torch.randn(n, generator=g0)
    w = torch.rand(n, generator=g0) * 3 if weighted else None
    f = F[:, 0]
    if obj == 0:
        g, h = f - y, torch.ones_like(f)
    elif obj == 1:
        g, h = torch.sign(f - y), torch.ones_like(f)
    elif obj == 2:
        r = f - y
        s = torch.sqrt(1 + r * r)
        g, h = r / s, 1 / (s * s * s)
    elif obj == 3:
        e = torch.exp(f)
        g, h = e - y, e * np.exp(0.7)
    elif obj == 4:
        p = torch.sigmoid(f)
        g, h = p - y, (p * (1 - p)).clamp_min(1e-16)
    if obj == 5:
        p = torch.softmax(F, 1)
        g = p - torch.nn.functional.one_hot(y.long(), C).float()
        h = (2 * p * (1 - p)).clamp_min(1e-16)
    else:
        g, h = g[:, None], h[:, None]
    if w is not None:
        g, h = g * w[:, None], h * w[:, None]
    gd, hd = K.grad_hess(F.to(dev), y.to(dev), None if w is None else w.to(dev), obj)
    torch.testing.assert_close(gd.cpu(), g, rtol=2e-6, atol=2e-6)
    torch.testing.assert_close(hd.cpu(), h, rtol=2e-6, atol=2e-6)


@pytest.mark.parametrize("raw", [True, "pair", False])
def test_hist_assemble(dev, raw):
    """Level histogram assembly kernel == the torch sequence (fixed-point scale(s), parent - sibling), and ==
    the CPU path of the same function (gloo ranks take it)."""
    g = torch.Generator().manual_seed(11)
    d, B, Kc = 7, 40, 2
    # 6 active nodes: siblings 0/1 (0 built), siblings 2/3 (3 built), 4 and 5 built without a sibling
    slot = np.array([0, -1, -1, 1, 2, 3], dtype=np.int64)
    parent = np.array([0, 0, 1, 1, -1, -1], dtype=np.int64)
    sib = np.array([1, 0, 3, 2, -1, -1], dtype=np.int64)
    if raw:
        Hb = torch.randint(-2 ** 40, 2 ** 40, (4, d, B, Kc), generator=g, dtype=torch.int64)
        scale = 2.0 ** 17 if raw is True else (2.0 ** 9, 2.0 ** 21)
        s0, s1 = K.raw_scales(scale)
        Hf = Hb.double()
        Hf[..., 0] /= s0
        Hf[..., 1] /= s1
    else:
        Hb = torch.randn(4, d, B, Kc, generator=g, dtype=torch.float64)
        scale, Hf = None, Hb
    prev = torch.randn(2, d, B, Kc, generator=g, dtype=torch.float64)
    ref = torch.empty(6, d, B, Kc, dtype=torch.float64)
    built = np.nonzero(slot >= 0)[0]
    ref[torch.from_numpy(built)] = Hf[torch.from_numpy(slot[built])]
    for a in np.nonzero(slot < 0)[0]:
        ref[a] = prev[parent[a]] - ref[sib[a]]
    out = K.hist_assemble(Hb.to(dev), scale, prev.to(dev), slot, parent, sib).cpu()
    assert torch.equal(out, ref)
    assert torch.equal(K.hist_assemble(Hb, scale, prev, slot, parent, sib), ref)


def test_hist_assemble_many_nodes(dev):
    """more than 65535 active nodes in one level (deep levels of many trees) -- the kernel strides
    nodes over the grid instead of rejecting the launch."""
    A = 70001
    g = torch.Generator().manual_seed(3)
    Hb = torch.randint(-2 ** 30, 2 ** 30, (A // 2 + 1, 1, 2, 2), generator=g, dtype=torch.int64)
    prev = torch.randn(A, 1, 2, 2, generator=g, dtype=torch.float64)
    slot = np.full(A, -1, dtype=np.int64)
    slot[0::2] = np.arange(len(slot[0::2]))
    sib = np.arange(A) + np.where(np.arange(A) % 2 == 0, 1, -1)
    sib[-1] = -1
    parent = np.arange(A) // 2
    ref = K.hist_assemble(Hb, 2.0 ** 5, prev, slot, parent, sib)
    out = K.hist_assemble(Hb.to(dev), 2.0 ** 5, prev.to(dev), slot, parent, sib).cpu()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("dtype,card", [(torch.int64, 7), (torch.int64, 300000), (torch.float64, 1000),
                                        (torch.float32, 5000), (torch.int32, 64)])
def test_hash_dense_ids_match_torch_unique(dev, dtype, card):
    """K16: hash-table dense ids == torch.unique's sorted inverse (incl. -0.0 == 0.0, INT64_MIN keys, and the
    overflow retry when the first table is too small)."""
    g = torch.Generator().manual_seed(card)
    x = torch.randint(-card, card, (400000,), generator=g).to(dtype)
    if dtype.is_floating_point:
        x = x / 7.0
        x[:5] = -0.0
    if dtype == torch.int64:
        x[7] = -(1 << 63)
    ids, G, vals = K.hash_dense_ids(x.to(dev))
    xr = torch.where(x == 0, torch.zeros_like(x), x) if dtype.is_floating_point else x
    uniq, inv = torch.unique(xr, return_inverse=True)
    assert G == uniq.numel()
    assert torch.equal(ids.cpu(), inv)
    assert torch.equal(vals.cpu(), uniq)


def test_dict_encode_matches_numpy(dev):
    """K17: device string dictionary encode == np.unique codes (nulls -> -1, empty strings, unicode)."""
    import pyarrow as pa
    rng = np.random.default_rng(0)
    words = np.array(["a", "", "bé", "zz", "Mark", "mark", "x" * 40] + [f"w{i}" for i in range(3000)], dtype=object)
    vals = words[rng.integers(0, len(words), 200000)]
    vals[::97] = None
    arr = pa.array(vals.tolist(), type=pa.string())
    codes, valid, dic = K.dict_encode(arr, dev)
    ok = np.array([v is not None for v in vals])
    uni, inv = np.unique(vals[ok].astype(str), return_inverse=True)
    assert dic.tolist() == uni.tolist()
    c = codes.cpu().numpy()
    assert (c[~ok] == -1).all() and np.array_equal(c[ok], inv)
    assert np.array_equal(valid.cpu().numpy(), ok)


def test_relational_on_hash_kernels_match_pandas(dev):
    """groupBy-count, avg, join and dropDuplicates through the K16/K17 device path == pandas."""
    import pandas as pd
    import cdnaml
    from cdnaml.sql import functions as F
    spark = cdnaml.SparkSession.builder.getOrCreate()
    rng = np.random.default_rng(3)
    n = 120000
    pdf = pd.DataFrame({"k": rng.integers(0, 5000, n), "s": rng.choice(["ann", "bob", "cé", None], n),
                        "v": rng.normal(size=n)})
    df = spark.createDataFrame(pdf)
    got = df.groupBy("k").count().orderBy("k").toPandas()
    ref = pdf.groupby("k").size().reset_index(name="count")
    assert got["k"].tolist() == ref["k"].tolist() and got["count"].tolist() == ref["count"].tolist()
    g2 = df.groupBy("s").agg(F.avg("v").alias("m")).toPandas().set_index("s")["m"]
    r2 = pdf.groupby("s", dropna=False)["v"].mean()
    for key, val in r2.items():
        k2 = None if (isinstance(key, float) and np.isnan(key)) else key
        assert g2.loc[g2.index.isna()].iloc[0] == pytest.approx(val) if k2 is None else \
            g2.loc[k2] == pytest.approx(val)
    dim = pd.DataFrame({"k": np.arange(0, 5000, 2), "name": [f"n{i}" for i in range(2500)]})
    j = df.join(spark.createDataFrame(dim), on="k").count()
    assert j == len(pdf.merge(dim, on="k"))
    assert df.dropDuplicates(["k", "s"]).count() == len(pdf.drop_duplicates(["k", "s"]))


@pytest.mark.parametrize("d,B", [(21, 40), (100, 40), (130, 64), (100, 80), (64, 32), (257, 17),
                                 (100, 100), (100, 256), (130, 200), (37, 256), (64, 128)])
def test_seg_hist_lane_matches_flat(dev, d, B, monkeypatch):
    """K5 lane-feature kernels (lanes own features, bin-major LDS plane) give exactly the int64 fixed-point
    sums of the flat (row, group)-pair kernel: partial 64-lane feature halves, two feature blocks (d > 128),
    B = 80, several chunks per segment and zero-weight records; 80 < B <= 256 runs the 64-feature
    quarter-wave variant (seg_hist_lane4_kernel, BP = 128 / 256)."""
    T, n = 6, 150000
    rng = np.random.default_rng(d * 7 + B)
    loc = rng.integers(0, 3, (T, n))
    w = rng.poisson(1.0, (T, n)).clip(0, 12)
    loc = np.where(w == 0, 0xFF, loc)
    codes = torch.from_numpy(((w << 8) | loc).astype(np.uint16).view(np.int16)).to(dev)
    tfirst = torch.from_numpy(np.arange(T, dtype=np.int32) * 3)
    slot_of = np.array([(t * 3 + k) if k < 2 else -1 for t in range(T) for k in range(3)], dtype=np.int32)
    slot_of[slot_of >= 0] = np.arange(int((slot_of >= 0).sum()))
    S = int((slot_of >= 0).sum())
    g = torch.Generator().manual_seed(d)
    X = torch.randn(n, d, generator=g)
    thr, nthr = _thresholds(X, B)
    bins, rm = K.binize(X.to(dev), thr.to(dev), nthr.to(dev), want_rm=True)
    if rm is None:
        rm = K.bins_row_major(bins)
    v1 = (torch.randn(n, generator=g) * 5).to(dev)
    sc = K.seg_scales(None, v1, 12, n)
    rec, _, _, _, sg = K.codes_compact(codes, tfirst, slot_of, S, None, v1, rec_scale=sc[1])
    sb = np.concatenate([sg, np.arange(S)[:, None]], 1)
    monkeypatch.setattr(K, "SEG_HIST_CHUNK", 20000)
    monkeypatch.setattr(K, "SEG_LANE", False)
    ref = K.seg_hist(bins, d, B, rec, None, None, None, sb, S, 12, sc, bins_rm=rm, rec=True, raw=True)
    monkeypatch.setattr(K, "SEG_LANE", True)
    got = K.seg_hist(bins, d, B, rec, None, None, None, sb, S, 12, sc, bins_rm=rm, rec=True, raw=True)
    assert got.dtype == torch.int64 and int(ref[..., 0].sum()) > 0
    assert torch.equal(got.cpu(), ref.cpu())


@pytest.mark.parametrize("d,B", [(100, 40), (100, 32), (84, 40), (92, 17), (96, 2)])
def test_seg10_rows_and_lane10_histogram(dev, d, B, monkeypatch):
    """seg10 rows (binize v5, rm_layout="s10") equal the torch layout reference K.bins_seg10, and the
    six-items-per-wave record histogram on them gives exactly the int64 sums of the flat (row, group)-pair
    kernel on the standard rows: ragged last trips, several chunks per segment, zero-weight records, d < 100
    (zero chunk bytes past d), B = 32 / 40 planes."""
    T, n = 6, 150011
    rng = np.random.default_rng(d * 11 + B)
    loc = rng.integers(0, 3, (T, n))
    w = rng.poisson(1.0, (T, n)).clip(0, 12)
    loc = np.where(w == 0, 0xFF, loc)
    codes = torch.from_numpy(((w << 8) | loc).astype(np.uint16).view(np.int16)).to(dev)
    tfirst = torch.from_numpy(np.arange(T, dtype=np.int32) * 3)
    slot_of = np.array([(t * 3 + k) if k < 2 else -1 for t in range(T) for k in range(3)], dtype=np.int32)
    slot_of[slot_of >= 0] = np.arange(int((slot_of >= 0).sum()))
    S = int((slot_of >= 0).sum())
    g = torch.Generator().manual_seed(d)
    X = torch.randn(n, d, generator=g)
    thr, nthr = _thresholds(X, B)
    bins, s10 = K.binize(X.to(dev), thr.to(dev), nthr.to(dev), want_rm=True, rm_layout="s10")
    assert s10 is not None and s10.shape == (n, 16, 8)
    assert torch.equal(s10, K.bins_seg10(bins, d))
    rm = K.bins_row_major(bins)
    v1 = (torch.randn(n, generator=g) * 5).to(dev)
    sc = K.seg_scales(None, v1, 12, n)
    rec, _, _, _, sg = K.codes_compact(codes, tfirst, slot_of, S, None, v1, rec_scale=sc[1])
    sb = np.concatenate([sg, np.arange(S)[:, None]], 1)
    monkeypatch.setattr(K, "SEG_HIST_CHUNK", 20000)
    monkeypatch.setattr(K, "SEG_LANE", False)
    ref = K.seg_hist(bins, d, B, rec, None, None, None, sb, S, 12, sc, bins_rm=rm, rec=True, raw=True)
    monkeypatch.setattr(K, "SEG_LANE", True)
    got = K.seg_hist(bins, d, B, rec, None, None, None, sb, S, 12, sc, bins_rm=s10, rec=True, raw=True, rm_s10=True)
    assert got.dtype == torch.int64 and int(ref[..., 0].sum()) > 0
    assert torch.equal(got.cpu(), ref.cpu())
    # level 0 without records: every row of non-zero weight is an item of its tree's root
    rcodes = torch.from_numpy(((w << 8) | np.where(w == 0, 0xFF, 0)).astype(np.uint16).view(np.int16)).to(dev)
    rrec, _, _, _, rsg = K.codes_compact(rcodes, torch.arange(T, dtype=torch.int32), np.arange(T, dtype=np.int32),
                                         T, None, v1, rec_scale=sc[1])
    rsb = np.concatenate([rsg, np.arange(T)[:, None]], 1)
    rref = K.seg_hist(bins, d, B, rrec, None, None, None, rsb, T, 12, sc, bins_rm=s10, rec=True, raw=True,
                      rm_s10=True)
    for t0, t1 in [(0, T), (2, 5)]:
        rgot = K.seg_hist_root(s10, d, B, rcodes, v1, sc[1], 12, t0, t1,
                               torch.zeros((t1 - t0, d, B, 2), dtype=torch.int64, device=dev))
        assert torch.equal(rgot.cpu(), rref[t0:t1].cpu())
    # one built node per tree below the root: local node 1 of every tree is slot 2 t + 1 of the record path
    cgot = K.seg_hist_codes(s10, d, B, codes, v1, sc[1], 12, np.arange(T), np.ones(T, np.int64), 0, T,
                            torch.zeros((T, d, B, 2), dtype=torch.int64, device=dev))
    assert torch.equal(cgot.cpu(), ref[1::2].cpu())


@pytest.mark.parametrize("d,B,off", [(100, 40, 0), (92, 17, 12345), (100, 32, 3)])
def test_root_histogram_draws_the_bootstrap(dev, d, B, off):
    """Level 0 with the Poisson draws fused into the root histogram kernel (lazy K.BootstrapCodes): the codes it
    writes equal the draws kernel's (misc.hip poisson_kernel, same Philox uniforms keyed by global row id + row
    offset, same tabulated CDF) and its int64 sums equal the root histogram over those codes."""
    T, n = 7, 100003
    g = torch.Generator().manual_seed(d + B)
    X = torch.randn(n, d, generator=g)
    thr, nthr = _thresholds(X, B)
    _, s10 = K.binize(X.to(dev), thr.to(dev), nthr.to(dev), want_rm=True, rm_layout="s10")
    v1 = (torch.randn(n, generator=g) * 3).to(dev)
    bound = K.poisson_max_draw(1.0)
    assert 8 <= bound <= 31
    sc = K.seg_scales(None, v1, bound, n)
    ref_codes = K.BootstrapCodes(T, n, 77, off, 1.0, dev)
    assert ref_codes.wmax() <= bound
    ref = K.seg_hist_root(s10, d, B, ref_codes.codes, v1, sc[1], bound, 0, T,
                          torch.zeros((T, d, B, 2), dtype=torch.int64, device=dev))
    lazy = K.BootstrapCodes(T, n, 77, off, 1.0, dev, lazy=True)
    assert lazy.pending and lazy.wmax() == bound
    got = K.seg_hist_codes(s10, d, B, lazy.codes, v1, sc[1], bound, np.arange(T), np.zeros(T, np.int64), 0, T,
                           torch.zeros((T, d, B, 2), dtype=torch.int64, device=dev), draw=lazy.draw_args())
    assert torch.equal(lazy.codes.cpu(), ref_codes.codes.cpu())
    assert torch.equal(got.cpu(), ref.cpu())


def test_fused_draws_grow_the_same_forest(dev, monkeypatch):
    """RandomForestRegressor with the bootstrap draws fused into the level-0 histogram equals the draws-kernel
    path bit for bit (forest digest)."""
    import cdnaml
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.utils.synthetic import forest_digest
    spark = cdnaml.SparkSession.builder.getOrCreate()
    g = torch.Generator(device=dev).manual_seed(4)
    X = torch.randn((300000, 100), generator=g, device=dev)
    y = (X[:, 0] * 2 - X[:, 1] + torch.sin(3 * X[:, 2])).double()
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
    calls = {"n": 0}
    orig = K.seg_hist_codes

    def counted(*a, **k):
        calls["n"] += k.get("draw") is not None
        return orig(*a, **k)
    monkeypatch.setattr(K, "seg_hist_codes", counted)
    digests = []
    for fused in (True, False):
        monkeypatch.setattr(K, "POISSON_FUSED", fused)
        digests.append(forest_digest(RandomForestRegressor(numTrees=20, maxDepth=5, maxBins=40, seed=3).fit(df)._forest))
    assert calls["n"] == 1 and digests[0] == digests[1]


@pytest.mark.parametrize("d,B", [(100, 256), (64, 256), (100, 100), (37, 129)])
def test_wide_codes_histogram_equals_records(dev, d, B):
    """Boosting levels with one built node per tree (80 < B <= 256) straight from the row codes
    (seg_hist_lane4_root_kernel) give the int64 sums of codes_compact records + the lane4 record histogram:
    bag weights 0/1/2, a non-root local node, slot-range slices."""
    T, n = 3, 150011
    rng = np.random.default_rng(d + B)
    w = rng.integers(0, 3, (T, n))
    loc = np.where(w == 0, 0xFF, rng.integers(0, 2, (T, n)))
    codes = torch.from_numpy(((w << 8) | loc).astype(np.uint16).view(np.int16)).to(dev)
    g = torch.Generator().manual_seed(d)
    X = torch.randn(n, d, generator=g)
    thr, nthr = _thresholds(X, B)
    bins, rm = K.binize(X.to(dev), thr.to(dev), nthr.to(dev), want_rm=True)
    if rm is None:
        rm = K.bins_row_major(bins)
    v1 = (torch.randn(n, generator=g) * 3).to(dev)
    sc = K.seg_scales(None, v1, 2, n)
    tfirst = torch.from_numpy(np.arange(T, dtype=np.int32) * 2)
    slot_of = np.array([t if k == 1 else -1 for t in range(T) for k in range(2)], dtype=np.int32)  # node 1 built
    rec, _, _, _, sg = K.codes_compact(codes, tfirst, slot_of, T, None, v1, rec_scale=sc[1])
    sb = np.concatenate([sg, np.arange(T)[:, None]], 1)
    ref = K.seg_hist(bins, d, B, rec, None, None, None, sb, T, 2, sc, bins_rm=rm, rec=True, raw=True)
    for s0, s1 in [(0, T), (1, 3)]:
        got = K.seg_hist_codes(rm, d, B, codes, v1, sc[1], 2, np.arange(T), np.ones(T, np.int64), s0, s1,
                               torch.zeros((s1 - s0, d, B, 2), dtype=torch.int64, device=dev))
        assert int(ref[s0:s1, ..., 0].sum()) > 0
        assert torch.equal(got.cpu(), ref[s0:s1].cpu())


@pytest.mark.parametrize("d,maxb,n,missing", [(100, 40, 100003, None), (64, 256, 5001, None), (8, 2, 77, None),
                                              (128, 32, 4099, None), (100, 40, 3001, -999.0),
                                              (100, 40, 3001, float("nan"))])
def test_binize_v5_matches_reference(dev, d, maxb, n, missing):
    """K4 binize v5 (wave = 64-row tile x 8-feature group, broadcast table reads, [64][17] row-major tile):
    column-major and padded row-major bins equal the CPU searchsorted reference -- categorical columns, NaN / +-inf,
    ragged last tile, 1..16 waves per block, 4-8 search steps, XGBoost missing values; the seg10 row layout
    equals the bins' repacking."""
    g = torch.Generator().manual_seed(d + maxb)
    X = torch.randn(n, d, generator=g) * 3
    X[:, 1] = torch.randint(0, 9, (n,), generator=g).float()
    thr, nthr = _thresholds(X, maxb)
    nthr[1] = -1
    X[5, 0] = float("nan")
    X[7, 2 % d] = float("inf")
    X[9, 3 % d] = -float("inf")
    if missing is not None and not math.isnan(missing):
        X[11:40, 4 % d] = missing
    ref = K.binize(X, thr, nthr, missing=missing)
    bins, rm = K.binize(X.to(dev), thr.to(dev), nthr.to(dev), missing=missing, want_rm=True)
    assert torch.equal(bins.cpu(), ref)
    G = (d + 7) // 8
    rmc = rm.cpu()
    assert rm is not None and torch.equal(rmc[:, :G], K.bins_row_major(ref)) and not rmc[:, G:].any()
    assert torch.equal(rm, K.bins_row_major(bins))
    if 80 < d <= 100 and maxb <= 40 and missing is None:
        b10, s10 = K.binize(X.to(dev), thr.to(dev), nthr.to(dev), want_rm=True, rm_layout="s10")
        assert torch.equal(b10, bins) and torch.equal(s10, K.bins_seg10(bins, d))


def test_fused_expressions_match_operator_path(dev, monkeypatch):
    """K18: every fusable expression gives exactly the operator-at-a-time torch result (values of valid rows and
    the validity mask), incl. nulls, NaN, division / modulo by zero, log of non-positives, casts with NaN,
    three-valued and/or, when chains with and without otherwise, round / floor / ceil / abs / signum."""
    import cdnaml
    from cdnaml.sql import fused
    from cdnaml.sql import functions as F
    spark = cdnaml.SparkSession.builder.getOrCreate()
    n = 20011
    g = torch.Generator().manual_seed(3)
    x = torch.randn(n, generator=g, dtype=torch.float64) * 5
    x[::17] = 0.0
    x[::29] = float("nan")
    y = torch.randn(n, generator=g, dtype=torch.float64).float()
    k = torch.randint(-3, 4, (n,), generator=g, dtype=torch.int32)
    pdf = pd.DataFrame({"x": x.numpy(), "y": y.numpy(), "k": k.numpy(),
                        "b": (k > 0).numpy(), "big": torch.randint(0, 10**6, (n,), generator=g).numpy()})
    pdf.loc[::13, "x"] = None
    pdf["k"] = pdf["k"].astype("Int32")
    pdf.loc[::11, "k"] = None
    df = spark.createDataFrame(pdf)
    x_, y_, k_, b_ = F.col("x"), F.col("y"), F.col("k"), F.col("b")
    exprs = {
        "arith": (x_ * 2.0 + y_) / (k_ - 1.0),
        "mod": (x_ + 0.5) % (k_ * 1.0),
        "logexp": F.exp(F.log(F.abs(x_) + 1.0)) - F.log1p(y_ * 1.0) + F.sqrt(x_ * 1.0) * F.log10(k_ * 1.0),
        "cmp3": ((x_ > 0) & (y_ < 0.5)) | ~(k_ == 2),
        "when": F.when(x_ > 1.0, x_ * 2.0).when(k_ < 0, y_ * 1.0).otherwise(-1.0) + 0.0,
        "when_null": F.when(b_, k_ * 1.0).when(x_ < 0, 3.0) * 2.0,
        "casts": (x_ * 3.0).cast("int") + (y_ * 1.0).cast("float") * 0.5,
        "casts2": ((x_ * 10.0).cast("long") + 1.0).cast("double") * k_.cast("double"),
        "round": F.round(x_ * 1.0, 2) + F.floor(y_ * 3.0) - F.ceil(x_ * 1.0) + F.signum(x_ * 1.0),
        "nulls": F.isnull(x_ * 1.0) | F.isnan(x_ * 2.0) | (F.col("big") * 1.0 > 5e5),
        "pow": F.pow(F.abs(x_) * 1.0, 0.5) + F.sin(x_ * 1.0) * F.cos(y_ * 1.0),
    }
    from cdnaml.models.util import local_batch
    b = local_batch(df, ["x", "y", "k", "b", "big"])
    for name, e in exprs.items():
        assert fused.can_fuse(e._expr, b), name          # the fused kernel really runs for each of them
        monkeypatch.setattr(fused, "FUSE", True)
        got = df.select(e.alias("r")).toPandas()["r"]
        monkeypatch.setattr(fused, "FUSE", False)
        ref = df.select(e.alias("r")).toPandas()["r"]
        assert got.isna().equals(ref.isna()), name
        gv, rv = got[~got.isna()].to_numpy(), ref[~ref.isna()].to_numpy()
        # device libm transcendentals may differ from torch's in the last ulp; arithmetic / masks are exact
        assert np.allclose(gv.astype(np.float64), rv.astype(np.float64), rtol=1e-12, atol=1e-300,
                           equal_nan=True), name


@pytest.mark.parametrize("T,n,offset,rate", [(20, 100003, 12, 1.0), (3, 4096, 0, 1.0), (5, 999, 7, 2.5)])
def test_bootstrap_codes_equal_codes_of_poisson_weights(dev, T, n, offset, rate):
    """K15 fused: the Poisson draws written straight as the engine's row codes (+ their max) equal codes_init of
    the uint8 multiplicities, and their weights() equal poisson_weights bit for bit."""
    w = K.poisson_weights(T, n, 31, offset, rate, device=dev)
    ref, wm = K.codes_init_max(w, T, n, dev)
    bc = K.BootstrapCodes(T, n, 31, offset, rate, dev)
    assert torch.equal(bc.codes, ref)
    assert bc.wmax() == wm == int(w.max())
    assert torch.equal(bc.weights(), w)


@pytest.mark.parametrize("n,offset,frac", [(1_000_003, 17, 1e-3), (5000, 0, 0.3), (1, 5, 0.999), (4096, 3, 1e-9)])
def test_sample_rows_equals_compacted_uniform(dev, n, offset, frac):
    """misc.hip sample_rows_kernel (one fused pass, ids claimed per wave, sorted after) == the materialised
    compact_mask(uniform(...) < frac) of the quantile sample."""
    ids = K.sample_rows(n, 0x5BD1E995 ^ 7, offset, 3, frac, dev)
    ref = K.compact_mask(K.uniform(n, 0x5BD1E995 ^ 7, offset, 3, device=dev) < frac)
    assert ids is not None and torch.equal(ids, ref)


def test_float_with_absmax(dev):
    """misc.hip cast_absmax_kernel: the fp32 copy and max |x| of an fp64 column (odd length: the scalar tail;
    a NaN surfaces as a NaN maximum, which packed_scale_global rejects)."""
    g = torch.Generator(device=dev).manual_seed(5)
    y = torch.randn(1_000_001, generator=g, device=dev, dtype=torch.float64) * 3
    y[77] = -41.5
    yf = K.float_with_absmax(y)
    assert torch.equal(yf, y.float())
    assert K._prefetched(yf, True) == float(y.float().abs().max()) == 41.5
    y[5] = float("nan")
    assert math.isnan(K._prefetched(K.float_with_absmax(y), True))
    z = K.float_with_absmax(torch.zeros(3, dtype=torch.float64, device=dev))
    assert K._prefetched(z, True) == 0.0


def test_heap_predict_double_store(dev):
    """predict_heap_kernel sums in fp64 (its fp32 store is the rounded fp64 result) and equals the int4-node
    kernel and the cpu reference bit for bit (the same fixed tree order), including a forest with shallow leaves
    (pass-through slots) and categorical splits."""
    import cdnaml
    from cdnaml.models.regression import RandomForestRegressor
    spark = cdnaml.SparkSession.builder.getOrCreate()
    g = torch.Generator(device=dev).manual_seed(2)
    X = torch.randn((20000, 12), generator=g, device=dev)
    y = (X[:, 0] - 2 * X[:, 3]).double()
    m = RandomForestRegressor(numTrees=6, maxDepth=4, seed=1).fit(
        spark.createDataFrameFromLocalTensors({"features": X, "label": y}))
    ha = m._forest.heap_arrays(X.device, "value")
    tw = torch.tensor(m._tree_w, dtype=torch.float64, device=dev)
    a = K.tree_predict_heap(X, ha[0], ha[1], tw, ha[2], 0.25, dtype=torch.float32)
    b = K.tree_predict_heap(X, ha[0], ha[1], tw, ha[2], 0.25, dtype=torch.float64)
    assert b.dtype == torch.float64 and torch.equal(b.float(), a)
    nodes, roots, vals, masks = m._forest.device_arrays(X.device, "value")
    base = torch.tensor([0.25], dtype=torch.float64, device=dev)
    c = K.tree_predict(X, nodes, roots, tw, vals, masks, 1, base)
    assert torch.equal(b, c)
    ref = K.tree_predict(X.cpu(), nodes.cpu(), roots.cpu(), tw.cpu(), vals.cpu(), masks.cpu(), 1, base.cpu())
    assert torch.equal(b.cpu(), ref)
    # categorical splits and leaves at several depths
    nodes2, roots2, vals2, masks2 = _random_forest_arrays(9, 5, 12, 1, 3)
    cat = nodes2[:, 0] < -1
    nodes2[cat, 0] = -(3 + 2)
    Xc = X.clone()
    Xc[:, 3] = torch.randint(0, 40, (X.shape[0],), generator=g, device=dev).float()
    f = _forest_from_arrays(nodes2, roots2, vals2, masks2)
    hs = f.heap_struct()
    assert hs is not None and hs[2] == 5
    heap = torch.from_numpy(K.pack_heap(hs[0], hs[1], hs[2])).to(dev)
    tw2 = torch.rand(9, dtype=torch.float64, generator=torch.Generator().manual_seed(4)).to(dev)
    got = K.tree_predict_heap(Xc, heap, hs[2], tw2, torch.from_numpy(hs[3]).to(dev), 0.0)
    n3, r3, v3, m3 = f.device_arrays(torch.device("cpu"))
    want = K.tree_predict(Xc.cpu(), n3, r3, tw2.cpu(), v3, m3, 1, None)
    assert torch.equal(got.cpu(), want)
    assert torch.equal(K.tree_predict(Xc, n3.to(dev), r3.to(dev), tw2, v3.to(dev), m3.to(dev), 1, None).cpu(), want)


def _forest_from_arrays(nodes, roots, vals, masks):
    """A host Forest from _random_forest_arrays' int4 node table (K = 1), with some leaves cut shallow."""
    from cdnaml.models.tree.engine import Forest
    nd = nodes.numpy()
    f = Forest(1)
    L = f.lists()
    mk = masks.numpy().view(np.uint32).reshape(-1, 8) if masks.numel() else np.zeros((0, 8), np.uint32)
    v = vals.numpy()
    for i, (a, b, l, r) in enumerate(nd.tolist()):
        shallow = a != -1 and i % 7 == 3  # turn some internal nodes into leaves (unreachable subtrees)
        leaf = a == -1 or shallow
        L["feat"].append(-1 if leaf else (a if a >= 0 else -a - 2))
        L["thr"].append(0.0 if leaf or a < 0 else float(np.array([b], np.int32).view(np.float32)[0]))
        L["bin"].append(0)
        L["left"].append(-1 if leaf else l)
        L["right"].append(-1 if leaf else r)
        L["catmask"].append(mk[b] if (not leaf and a < -1) else np.zeros(8, np.uint32))
        L["is_cat"].append(bool(not leaf and a < -1))
        L["value"].append(np.array([v[b] if a == -1 else 0.5 * i], np.float64))
        L["weight"].append(1.0)
        L["gain"].append(0.0)
        L["impurity"].append(0.0)
        L["depth"].append(0)
    f.roots.extend(roots.tolist())
    return f



def test_shifted_f32(dev):
    """misc.hip cast_absmax_kernel with a device shift: (y - s).float() with the subtraction in fp64 (odd length:
    the scalar tail)."""
    g = torch.Generator(device=dev).manual_seed(6)
    y = 1e5 + torch.randn(100_001, generator=g, device=dev, dtype=torch.float64) * 3
    s = y[:1024].mean().reshape(1)
    assert torch.equal(K.shifted_f32(y, s), (y - s).float())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4096, 1001])
def test_codes_to_nodes_matches_torch(n):
    """seg.hip codes_to_nodes_kernel (vectorised when n % 4 == 0, scalar otherwise) == the torch decode."""
    from cdnaml.ops import kernels as K
    g = torch.Generator().manual_seed(n)
    T = 5
    loc = torch.randint(0, 256, (T, n), generator=g)
    w = torch.randint(0, 4, (T, n), generator=g)
    codes = ((w << 8) | loc).to(torch.int16)
    tfirst = torch.tensor([0, 7, 300, 301, 900], dtype=torch.int32)
    node, wd = K.decode_codes(codes.cuda(), tfirst)
    ids = tfirst[:, None].long() + loc
    ref = torch.where((loc == K.CODE_DONE) | (w == 0), torch.full_like(ids, -1), ids)
    assert torch.equal(node.cpu().long(), ref)
    assert torch.equal(wd.cpu().long(), w)


@pytest.mark.gpu
@pytest.mark.parametrize("d,k", [(100, 33), (7, 3), (300, 17), (64, 63), (1, 1)])
def test_feature_masks_match_host(d, k):
    """misc.hip feature_masks_kernel == the host draw of ForestTrainer._feature_masks (k smallest splitmix64 hashes
    of base + f * C per node, as bit words)."""
    import numpy as np
    from cdnaml.models.tree.engine import _splitmix64
    from cdnaml.ops import kernels as K
    rng = np.random.default_rng(d * 1000 + k)
    A = 777
    base = rng.integers(0, 2 ** 63, size=A, dtype=np.int64).astype(np.uint64) * np.uint64(2) + np.uint64(1)
    with np.errstate(over="ignore"):
        h = _splitmix64(base[:, None] + np.arange(d, dtype=np.uint64)[None, :] * np.uint64(0xD6E8FEB86659FD93))
    feats = np.argpartition(h, k - 1, axis=1)[:, :k]
    words = np.zeros((A, (d + 31) // 32), dtype=np.uint32)
    f = feats.reshape(-1)
    np.bitwise_or.at(words, (np.repeat(np.arange(A), k), f >> 5), np.uint32(1) << (f & 31).astype(np.uint32))
    got = K.feature_masks(base, d, k, torch.device("cuda")).cpu().numpy().view(np.uint32)
    assert np.array_equal(got, words)
