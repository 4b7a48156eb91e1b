"""Binning for the tree learner: per-feature split thresholds from a global quantile
sample (Spark findSplits semantics; Philox-sampled rows keyed by the global row id, all-gathered, so the bins do
not depend on the GPU count), and the uint8 bins of this rank's rows -- column groups [G][n][8] plus the row-major
copy the segment histograms gather (seg10 rows at d <= 100, B <= 40).  ``X`` may be resident or a
:class:`ChunkedRows` stream (out-of-core fits: the sample and the bins are built chunk by chunk)."""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import torch

from ...ops import kernels as K
from ...utils import tracing as _tr
from ..util import IllegalArgumentException

# binning queued on the quantile kernel's device thresholds, checked on the host behind it
SPEC_THRESHOLDS = True
# one-rank quantile sample gathered on the device behind the Philox selection (no host count round trip)
SAMPLE_FUSED = True
# free device memory kept back when building the boosting partition's feature-major bins copy
FM_HEADROOM = 4 << 30


# ============================================================ binning (K3/K4)
@dataclass
class BinnedData:
    X: torch.Tensor
    bins: torch.Tensor
    thresholds: np.ndarray            # [d, B-1] float64 raw thresholds
    nthr: np.ndarray                  # [d] int (-1 categorical)
    categorical: Dict[int, int]
    n_local: int
    n_global: int
    row_offset: int
    d: int
    B: int
    missing_bin: bool = False         # bin 0 holds missing values (XGBoost sparsity-aware splits)
    bins_rm: Optional[torch.Tensor] = None  # lazily built row-major copy [n, G, 8] (segment-mode histograms)
    bins_s10: Optional[torch.Tensor] = None  # seg10 row layout [n, 16, 8] written by binize (K.bins_seg10)
    bins_fm: Optional[torch.Tensor] = None   # lazily built feature-major byte copy [G * 8, n] (boosting partitions)
    source_ref: Optional[object] = None      # weakref to the frame's feature tensor of the latest fit (FitBins)

    def row_major_bins(self) -> torch.Tensor:
        if self.bins_rm is None:
            self.bins_rm = K.bins_row_major(self.bins)
        return self.bins_rm

    def feature_major_bins(self) -> Optional[torch.Tensor]:
        """[G * 8, n] uint8: byte f * n + r is row r's bin of feature f (built once, kept for the fit's rounds and
        released by ``release_fit_copies`` when the boosting fit ends).  None when the device cannot hold the
        second copy with FM_HEADROOM to spare (the partition then gathers from the [G][n] words: ADVICE r5, a
        1e8 x 100 fit's copy is ~10 GB next to the bins and usually the row-major copy)."""
        if self.bins_fm is None:
            G, n, _ = self.bins.shape
            if self.bins.is_cuda:
                free, _ = torch.cuda.mem_get_info(self.bins.device)
                if free < G * 8 * n + FM_HEADROOM:
                    return None
            self.bins_fm = self.bins.permute(0, 2, 1).reshape(G * 8, n).contiguous()
        return self.bins_fm

    def release_fit_copies(self) -> None:
        """Drop the per-fit feature-major copy (the cached binned data outlives the fit: CV / tuning reuse it)."""
        self.bins_fm = None

    def record_rows(self):
        """(rows, is_seg10) for the record histograms: the seg10 copy when binize wrote one, else the standard
        row-major copy."""
        if self.bins_s10 is not None:
            return self.bins_s10, True
        return self.row_major_bins(), False


def _seg10_ok(X: torch.Tensor, d: int, max_bins: int) -> bool:
    return K.SEG10 and X.is_cuda and 80 < d <= 100 and d % 4 == 0 and max_bins <= 40


def find_thresholds(sample: np.ndarray, d: int, max_bins: int, categorical: Dict[int, int]):
    """Per-feature split thresholds from a (global) sample (Spark findSplits semantics)."""
    thr = np.zeros((d, max(max_bins - 1, 1)), dtype=np.float64)
    nthr = np.zeros(d, dtype=np.int32)
    for f in range(d):
        if f in categorical:
            nthr[f] = -1
            continue
        col = sample[:, f]
        col = col[~np.isnan(col)]
        if col.size == 0:
            continue
        vals, counts = np.unique(col, return_counts=True)
        if len(vals) <= 1:
            continue
        if len(vals) <= max_bins:
            cand = (vals[:-1] + vals[1:]) / 2.0
        else:
            cum = np.cumsum(counts)
            total = cum[-1]
            targets = total * np.arange(1, max_bins) / max_bins
            idx = np.searchsorted(cum, targets, side="left")
            idx = np.unique(np.clip(idx, 0, len(vals) - 2))
            cand = (vals[idx] + vals[idx + 1]) / 2.0
        cand = np.unique(cand)[: max_bins - 1]
        thr[f, : len(cand)] = cand
        nthr[f] = len(cand)
    return thr, nthr


def find_thresholds_t(samp: torch.Tensor, max_bins: int, categorical: Dict[int, int]):
    """``find_thresholds`` on a [s, d] float64 tensor, vectorised over features (runs on the sample's device).

    Features with more distinct values than ``max_bins`` (the common continuous case) take the batched
    quantile path: one sort of the whole sample, the quantile positions, and a batched searchsorted for
    the next distinct value.  Categorical / few-distinct / empty features fall back to the per-feature host
    code on their (already sorted) column.  Bit-identical to ``find_thresholds``.
    """
    s, d = samp.shape
    thr = np.zeros((d, max(max_bins - 1, 1)), dtype=np.float64)
    nthr = np.zeros(d, dtype=np.int32)
    if s == 0 or d == 0:
        for f in categorical:
            nthr[f] = -1
        return thr, nthr
    dev = samp.device
    q = K.quantile_thresholds(samp, max_bins)
    if q is not None:
        # one K3 kernel (sort in LDS + candidates + de-dup per feature block) instead of ~20 torch launches
        qthr, qn, kdist, S = q
        fast = kdist > max_bins
        for f in categorical:
            fast[f] = False
        thr[fast], nthr[fast] = qthr[fast], qn[fast]
        slow = np.nonzero(~fast)[0].tolist()
        if slow:
            cols = S[slow].t().cpu().numpy()
            t2, n2 = find_thresholds(cols, len(slow), max_bins,
                                     {i: categorical[f] for i, f in enumerate(slow) if f in categorical})
            thr[slow], nthr[slow] = t2, n2
        return thr, nthr
    S = torch.sort(samp.t().contiguous(), dim=1).values          # [d, s], NaN last
    nn = (~torch.isnan(S)).sum(1)                                 # non-NaN count per feature
    Sf = torch.where(torch.isnan(S), torch.full_like(S, float("inf")), S)
    ar = torch.arange(s, device=dev)
    valid = ar[None, :] < nn[:, None]
    newv = torch.ones_like(valid)
    newv[:, 1:] = Sf[:, 1:] != Sf[:, :-1]
    k = (newv & valid).sum(1)                                     # distinct non-NaN values
    cat = torch.zeros(d, dtype=torch.bool, device=dev)
    if categorical:
        cat[torch.tensor(sorted(categorical), device=dev)] = True
    fast = (k > max_bins) & ~cat
    if max_bins > 1 and bool(fast.any()):
        j = torch.arange(1, max_bins, device=dev, dtype=torch.int64)
        tgt = (nn[:, None] * j[None, :]).double() / max_bins      # same operations as the host code
        pos = (torch.ceil(tgt).long() - 1).clamp_min(0)
        pos = torch.minimum(pos, (nn - 1).clamp_min(0)[:, None])
        v = Sf.gather(1, pos)
        vmax = Sf.gather(1, (nn - 1).clamp_min(0)[:, None])
        first_max = torch.searchsorted(Sf, vmax, right=False)
        prev_max = Sf.gather(1, (first_max - 1).clamp_min(0))
        v = torch.where(v == vmax, prev_max, v)                  # idx clipped to len(vals) - 2
        nxt = Sf.gather(1, torch.searchsorted(Sf, v, right=True).clamp_max(s - 1))
        cand = ((v + nxt) / 2.0).cpu().numpy()
        # per feature np.unique of a nondecreasing row == drop repeats, for all features at once
        fr = torch.nonzero(fast).flatten().cpu().numpy()
        cf = cand[fr]
        keep = np.ones(cf.shape, dtype=bool)
        keep[:, 1:] = (cf[:, 1:] != cf[:, :-1]) & ~(np.isnan(cf[:, 1:]) & np.isnan(cf[:, :-1]))
        col = np.cumsum(keep, 1) - 1
        rows = np.broadcast_to(fr[:, None], cf.shape)
        thr[rows[keep], col[keep]] = cf[keep]
        nthr[fr] = keep.sum(1)
    slow = torch.nonzero(~fast).flatten().tolist()
    if slow:
        cols = S[slow].t().cpu().numpy()
        t2, n2 = find_thresholds(cols, len(slow), max_bins,
                                 {i: categorical[f] for i, f in enumerate(slow) if f in categorical})
        thr[slow], nthr[slow] = t2, n2
    return thr, nthr


class ChunkedRows:
    """This rank's feature rows as a re-iterable stream of ``(row0, X_chunk [m, d] f32)`` (out-of-core fits,
    SURVEY §5.7): the quantile sample and the binning read the chunks one at a time, so fp32 X is never
    resident -- only its uint8 bins are.  ``it_fn()`` starts a new pass; chunks are transient (the source may
    reuse their buffers once the work queued on them has run).  ``host_it_fn`` (optional) yields the same
    ``(row0, X_chunk)`` from HOST memory, without any copy: the quantile sample gathers its few rows there."""

    def __init__(self, it_fn, n: int, d: int, device, host_it_fn=None):
        self.it_fn, self.n, self.d, self.device = it_fn, int(n), int(d), torch.device(device)
        self.host_it_fn = host_it_fn
        self.shape = (self.n, self.d)
        self.is_cuda = self.device.type == "cuda"

    def __iter__(self):
        return iter(self.it_fn())


def _global_sample(session, X, max_bins: int, seed: int, row_offset: int, n_global: int, fused: bool = False):
    """Rows sampled by Philox keyed on the GLOBAL row id (the same rows whatever the GPU count), gathered
    from every rank: the split-candidate sample (a row set: its order is not defined).  ``X`` may be a
    :class:`ChunkedRows` stream (the same rows, sampled chunk by chunk).

    fused (one rank, resident fp32 X on the GPU): ``(samp, ok)`` -- the sample as fp64 rows padded with NaN rows to
    a fixed capacity, with no host round trip (``K.sample_gather``: the quantile kernel counts non-NaN values only,
    so the thresholds are the exact sample's); ``ok()`` is False in the (12-sigma) case the capacity overflowed,
    then the caller takes the exact sample.  Otherwise the sample itself."""
    comm = session.comm
    n = X.shape[0]
    target = max(max_bins * max_bins, 10000)
    frac = min(1.0, target / max(n_global, 1))
    if fused and SAMPLE_FUSED and frac < 1.0 and not comm.distributed and not isinstance(X, ChunkedRows):
        r = K.sample_gather(X, seed ^ 0x5BD1E995, row_offset, 3, frac)
        if r is not None:
            return r
    if isinstance(X, ChunkedRows) and X.host_it_fn is not None and frac < 1.0:
        # the sampled rows (the same Philox draws on the device) gathered from the host chunks: a few thousand
        # rows cross PCIe instead of the whole frame
        parts = []
        for r0, Xh in X.host_it_fn():
            u = K.uniform(Xh.shape[0], seed ^ 0x5BD1E995, row_offset + r0, 3, device=X.device)
            ih = K.compact_mask(u < frac).cpu()
            parts.append(Xh.index_select(0, ih).float().to(X.device))
        samp = torch.cat(parts) if parts else torch.zeros((0, X.d), dtype=torch.float32, device=X.device)
    elif isinstance(X, ChunkedRows):
        parts = []
        for r0, Xc in X:
            if frac < 1.0:
                u = K.uniform(Xc.shape[0], seed ^ 0x5BD1E995, row_offset + r0, 3, device=Xc.device)
                parts.append(Xc[K.compact_mask(u < frac)].float())
            else:
                parts.append(Xc.float().clone())
        samp = torch.cat(parts) if parts else torch.zeros((0, X.d), dtype=torch.float32, device=X.device)
    elif frac < 1.0:
        # the quantile thresholds depend on the sample's values only (each column is sorted): the rows are
        # gathered in the kernel's arbitrary order, no sort of the ids
        idx = K.sample_rows(n, seed ^ 0x5BD1E995, row_offset, 3, frac, X.device, ordered=False) \
            if X.is_cuda and n else None
        if idx is None:
            u = K.uniform(n, seed ^ 0x5BD1E995, row_offset, 3, device=X.device)
            idx = K.compact_mask(u < frac)
        samp = X[idx]
    else:
        samp = X
    if comm.distributed:
        samp = torch.cat(comm.all_gather_varlen(samp.contiguous()))
    return samp


class _Once:
    """A callable run at most once (None: nothing)."""

    def __init__(self, fn):
        self.fn = fn

    def __call__(self):
        fn, self.fn = self.fn, None
        if fn is not None:
            fn()


def make_binned(session, X: torch.Tensor, categorical: Dict[int, int], max_bins: int, seed: int,
                row_offset: int, n_global: int, missing: Optional[float] = None, before_binize=None) -> BinnedData:
    """:func:`_make_binned`, reused across the trials of one hyperparameter search (bincache.scope(), entered by
    fmin; never outside one).

    before_binize(): run once, right before the binning kernel is queued (after the quantile sample and the
    thresholds), or after a cache hit -- the caller's side-stream work that should overlap the memory-bound
    binning rather than the latency-bound sample / sort kernels (the bootstrap draws)."""
    from . import bincache
    hook = _Once(before_binize)
    if isinstance(X, ChunkedRows):  # streamed: no content fingerprint (X is never resident)
        data = _make_binned(session, X, categorical, max_bins, seed, row_offset, n_global, missing, hook)
    else:
        data = bincache.cached(
            lambda: (bincache.fingerprint(X), tuple(sorted(categorical.items())), int(max_bins), int(seed),
                     int(row_offset), int(n_global), None if missing is None else float(missing), str(X.device)),
            lambda: _make_binned(session, X, categorical, max_bins, seed, row_offset, n_global, missing, hook),
            comm=session.comm)
    hook()
    return data


def _binize_src(X, thr, nthr, missing=None, want_rm=False, rm_layout="std"):
    """K.binize of a tensor, or of a ChunkedRows stream chunk by chunk into full-size bins (and row copy)."""
    if not isinstance(X, ChunkedRows):
        return K.binize(X, thr, nthr, missing=missing, want_rm=want_rm, rm_layout=rm_layout)
    n, d = X.shape
    G = (d + 7) // 8
    bins = torch.empty((G, n, 8), dtype=torch.uint8, device=X.device)
    rm = None
    if want_rm and X.is_cuda:
        s10 = rm_layout == "s10"
        Gs = 16 if (s10 or (K.BINS_RM_PAD and G <= 16)) else G
        rm = torch.empty((n, Gs, 8), dtype=torch.uint8, device=X.device)
    rm_ok = rm is not None
    for r0, Xc in X:
        res = K.binize(Xc, thr, nthr, missing=missing, want_rm=rm_ok, rm_layout=rm_layout,
                       out_full=(bins, rm), row0=r0)
        rm_ok = rm_ok and res[1] is not None
    if want_rm and not rm_ok:  # a chunk took a kernel without the row copy: rebuilt from the bins on demand
        rm = None if rm_layout != "s10" or not X.is_cuda else K.bins_seg10(bins, d)
    return bins, (rm if want_rm else None)


def _make_binned(session, X, categorical: Dict[int, int], max_bins: int, seed: int,
                 row_offset: int, n_global: int, missing: Optional[float] = None, before_binize=None) -> BinnedData:
    """Global-sample quantile thresholds + device binning.

    ``missing`` (XGBoost semantics, ML 11:67 ``missing=0``): NaN and values equal
    to ``missing`` go to a dedicated bin 0; the remaining ``max_bins - 1`` bins
    hold the observed values, so every split can route missing rows either way.
    """
    d = X.shape[1]
    before_binize = before_binize if before_binize is not None else (lambda: None)
    if missing is not None:
        # thresholds of the observed values from the (missing -> NaN) global sample; the binning kernel maps
        # missing values to -inf -> bin 0 on the fly (no masked copies of the full matrix)
        samp = _global_sample(session, X, max_bins - 1, seed, row_offset, n_global)
        sm = torch.isnan(samp) if math.isnan(missing) else (torch.isnan(samp) | (samp == float(missing)))
        samp = torch.where(sm, torch.full_like(samp, float("nan")), samp)
        if max_bins > 2:
            with _tr.span("tree.find_thresholds"):
                ithr, inthr = find_thresholds_t(samp.double(), max_bins - 1, {})
        else:
            ithr, inthr = np.zeros((d, 0)), np.zeros(d, dtype=np.int32)
        thr = np.concatenate([np.full((d, 1), -np.finfo(np.float32).max), ithr], 1)
        nthr = inthr + 1
        thr_t = torch.from_numpy(thr.astype(np.float32)).to(X.device)
        before_binize()
        with _tr.span("tree.binize"):
            bins, rm = _binize_src(X, thr_t, torch.from_numpy(nthr).to(X.device), missing=float(missing),
                                   want_rm=True)
        return BinnedData(_resident(X), bins, thr, nthr, {}, X.shape[0], n_global, row_offset, d, max_bins, True,
                          rm)
    for f, k in categorical.items():
        if k > max_bins:
            raise IllegalArgumentException(
                f"requirement failed: DecisionTree requires maxBins (= {max_bins}) to be at least as large as the "
                f"number of values in each categorical feature, but categorical feature {f} has {k} values. "
                f"Consider removing this and other categorical features with a large number of values, or add "
                f"more training examples.")
    if max_bins > 256:
        raise IllegalArgumentException("maxBins must be <= 256 on this engine (uint8 bins)")
    n = X.shape[0]
    spec = SPEC_THRESHOLDS and not categorical and X.is_cuda and not isinstance(X, ChunkedRows)
    samp = _global_sample(session, X, max_bins, seed, row_offset, n_global, fused=spec)
    samp, samp_ok = samp if isinstance(samp, tuple) else (samp, lambda: True)
    s10 = _seg10_ok(X, d, max_bins)
    if spec:
        # the binning queued straight on the K3 kernel's device thresholds; the host checks behind it that every
        # feature had more than max_bins distinct sample values (then the thresholds are exactly the host path's)
        # -- no device -> host -> device round trip between the quantile kernel and the binning
        with _tr.span("tree.find_thresholds"):
            q = K.quantile_thresholds_dev(samp, max_bins)
        if q is not None:
            thr_d, nthr_d, pend = q
            before_binize()
            with _tr.span("tree.binize"):
                bins, rm = K.binize(X, thr_d, nthr_d, want_rm=True, rm_layout="s10" if s10 else "std")
            thr, ints = pend.get()
            if samp_ok() and bool((ints[1] > max_bins).all()):
                thr, nthr = thr.copy(), ints[0].copy()
                if s10:
                    return BinnedData(X, bins, thr, nthr, {}, n, n_global, row_offset, d, max_bins, False, None, rm)
                return BinnedData(X, bins, thr, nthr, {}, n, n_global, row_offset, d, max_bins, False, rm)
            del bins, rm  # a feature with few distinct values: the host path below, then bin again
    if not samp_ok():  # the fused sample's capacity overflowed: the exact sample
        samp = _global_sample(session, X, max_bins, seed, row_offset, n_global)
    with _tr.span("tree.find_thresholds"):
        thr, nthr = find_thresholds_t(samp.double(), max_bins, categorical)
    thr_t = torch.from_numpy(thr.astype(np.float32)).to(X.device)
    nthr_t = torch.from_numpy(nthr).to(X.device)
    before_binize()
    with _tr.span("tree.binize"):
        # the row-major copy (segment histograms' row gathers) comes out of the same kernel
        bins, rm = _binize_src(X, thr_t, nthr_t, want_rm=True, rm_layout="s10" if s10 else "std")
    if s10:
        return BinnedData(_resident(X), bins, thr, nthr, dict(categorical), n, n_global, row_offset, d, max_bins,
                          False, None, rm)
    return BinnedData(_resident(X), bins, thr, nthr, dict(categorical), n, n_global, row_offset, d, max_bins,
                      False, rm)


def _resident(X):
    """BinnedData.X: the feature matrix, or None for a streamed (out-of-core) source."""
    return None if isinstance(X, ChunkedRows) else X


from ...ops import tune as _tune  # noqa: E402  (CDNAML_TUNE overrides of the constants above)
_tune.apply(__import__(__name__, fromlist=["_"]))
