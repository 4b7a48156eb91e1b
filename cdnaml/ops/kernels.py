"""Tensor-level entry points for every native kernel (SURVEY §2.10 K1–K15).

Each op dispatches on the device of its inputs:

* device tensors (ROCm/HIP) -> the hand-written gfx950 kernel in
  ``csrc/kernels`` via :mod:`cdnaml.ops._lib` (fails loudly if the library
  cannot be built/loaded);
* CPU tensors -> a plain PyTorch reference implementation of the same op.
  These references define the semantics and are the oracles of the GPU
  numerics tests (tests/test_kernels_gpu.py).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib
from . import philox as _philox


from ._base import _TORCH_DT, _native, _ptr, _stream, upload  # noqa: F401


# --------------------------------------------------------------------- K1
def gram(X: torch.Tensor, y: Optional[torch.Tensor] = None, shift: Optional[torch.Tensor] = None,
         yshift: float = 0.0, bf16: bool = False, fp64: bool = False) -> torch.Tensor:
    """Return A^T A (float64, (d+2)x(d+2)) for A = [X - shift | 1 | y - yshift].

    Column d is the intercept column of ones; column d+1 is y (zeros if None).
    fp64: the fp32 augmented matrix multiplied in fp64 by the library GEMM (the CPU path's arithmetic) instead of
    the K1 MFMA kernel.
    """
    n, d = X.shape
    if X.dtype == torch.float64:
        # Spark's Double vectors (course scale): the augmented matrix is formed and multiplied in fp64 as is --
        # no fp32 rounding of the features (the shift is the caller's fp32-rounded value, used exactly)
        A = torch.empty((n, d + 2), dtype=torch.float64, device=X.device)
        A[:, :d] = X if shift is None else X - shift.double()
        A[:, d] = 1.0
        A[:, d + 1] = 0.0 if y is None else (y.double() - yshift)
        return A.T @ A
    if X.dtype != torch.float32:
        X = X.float()
    if _native(X) and d + 2 <= 512 and not fp64:
        X = X if X.stride(1) == 1 else X.contiguous()
        y32 = None if y is None else y.float().contiguous()
        sh = None if shift is None else shift.float().contiguous()
        L = _lib.lib()
        ws_n = L.cdna_gram_workspace(n, d, int(bf16))
        ws = torch.empty(max(ws_n, 1), dtype=torch.float32, device=X.device)
        out = torch.zeros((d + 2, d + 2), dtype=torch.float64, device=X.device)
        _lib.check(L.cdna_gram(_ptr(X), n, d, X.stride(0), _ptr(y32), _ptr(sh), float(yshift), _ptr(out), _ptr(ws),
                               int(bf16), _stream(X.device)), "cdna_gram")
        return out
    A = torch.empty((n, d + 2), dtype=torch.float32, device=X.device)
    A[:, :d] = X if shift is None else X - shift.float()
    A[:, d] = 1.0
    A[:, d + 1] = 0.0 if y is None else (y.float() - yshift)
    if bf16:
        A = A.to(torch.bfloat16)
    A = A.double()
    return A.T @ A


# -------------------------------------------------------------------- K15
def uniform(n: int, seed: int, offset: int = 0, stream: int = 0, device=None) -> torch.Tensor:
    """Philox uniform doubles keyed by (seed, offset+i, stream)."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    if device.type == "cuda":
        out = torch.empty(n, dtype=torch.float64, device=device)
        _lib.check(_lib.lib().cdna_uniform(_ptr(out), n, seed, int(offset), int(stream) & 0xFFFFFFFF,
                                           _stream(device)), "cdna_uniform")
        return out
    return torch.from_numpy(_philox.uniform(n, seed, int(offset), int(stream)))


def normal32_(out: torch.Tensor, seed: int, offset: int = 0, stream: int = 0) -> torch.Tensor:
    """Fill the contiguous fp32 tensor ``out`` with standard normals for global elements offset..offset+numel-1
    (Philox quads, Box-Muller; ``normal_f32_kernel``).  CPU: the numpy oracle ``philox.normal32``."""
    if out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("normal32_ needs a contiguous float32 tensor")
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    if out.is_cuda:
        _lib.check(_lib.lib().cdna_normal_f32(_ptr(out), out.numel(), seed, int(offset), int(stream) & 0xFFFFFFFF,
                                              _stream(out.device)), "cdna_normal_f32")
        return out
    out.view(-1).copy_(torch.from_numpy(_philox.normal32(out.numel(), seed, int(offset), int(stream))))
    return out


def poisson_weights(T: int, n: int, seed: int, offset: int, rate: float, device=None) -> torch.Tensor:
    """uint8 [T, n] Poisson(rate) bootstrap multiplicities, tree t on stream 0x100+t."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    if device.type == "cuda":
        out = torch.empty((T, n), dtype=torch.uint8, device=device)
        _lib.check(_lib.lib().cdna_poisson(_ptr(out), T, n, seed, int(offset), float(rate), None, None, 0,
                                           _stream(device)), "cdna_poisson")
        return out
    return torch.from_numpy(_philox.poisson(T, n, seed, int(offset), float(rate)))


POISSON_CODES = True


# where the forest's bootstrap draws run when the level-0 root histogram cannot draw them itself (POISSON_FUSED):
# "main" -- in series before the binning, "side" -- on the side stream at the same point (profiles/r4/prologue_ab.md).
# (An "auto" placement that started small shards' draws on the side stream with the fit measured 17.6 vs 17.5 ms at
# the 8-GPU point's per-rank shape against the fused draws, and was removed.)
POISSON_STREAM = "main"


def poisson_max_draw(rate: float) -> int:
    """The largest bootstrap weight the tabulated Poisson draws can produce at ``rate`` (-1: no static bound)."""
    return int(_lib.lib().cdna_poisson_max_draw(float(rate)))


# level 0 of a bootstrapped forest draws its Poisson weights inside the root histogram kernel (seg.hip RootDraw)
# instead of a draws kernel in series ahead of it
POISSON_FUSED = True


class BootstrapCodes:
    """Poisson bootstrap draws written straight as the tree engine's row codes (GPU): ``codes`` [T, n] int16
    (weight << 8 | 0, 0xFF for weight 0 -- codes_init's format) and the largest weight, copied to the host behind
    the kernel (``wmax()`` waits for that copy only).  ``weights()`` derives the uint8 multiplicities for the
    paths that need them (bit-identical to poisson_weights).

    lazy: nothing is launched yet when the draws have a static bound (``poisson_max_draw``): the trainer's level-0
    root histogram draws and writes the codes itself (``draw_args`` / ``mark_drawn``), any other first reader calls
    ``materialize`` (the draws kernel); ``wmax()`` is then the static bound."""

    def __init__(self, T: int, n: int, seed: int, offset: int, rate: float, device, grid_blocks: int = 0,
                 lazy: bool = False):
        dev = torch.device(device)
        self.T, self.n, self.seed, self.offset, self.rate, self.dev = T, n, int(seed), int(offset), float(rate), dev
        self.codes = torch.empty((T, n), dtype=torch.int16, device=dev)
        self._bound = poisson_max_draw(rate) if lazy else -1
        self.pending = self._bound >= 1
        self._wmax = None
        if not self.pending:
            self._launch(grid_blocks)

    def _launch(self, grid_blocks: int = 0) -> None:
        wm = torch.zeros(1, dtype=torch.int32, device=self.dev)
        _lib.check(_lib.lib().cdna_poisson(None, self.T, self.n, self.seed & 0xFFFFFFFFFFFFFFFF, self.offset,
                                           self.rate, _ptr(self.codes), _ptr(wm), int(grid_blocks),
                                           _stream(self.dev)), "cdna_poisson(codes)")
        self._wmax = _PendingScalar(wm, torch.cuda.current_stream(self.dev))

    def draw_args(self):
        """(seed, row offset, rate) for a kernel that draws the pending codes itself, else None."""
        return (self.seed, self.offset, self.rate) if self.pending else None

    def mark_drawn(self) -> None:
        self.pending = False

    def materialize(self) -> None:
        if self.pending:
            self._launch()
            self.pending = False

    def wmax(self) -> int:
        if self._bound >= 1:
            return self._bound
        return max(1, int(self._wmax.get()))

    def weights(self) -> torch.Tensor:
        self.materialize()
        return ((self.codes.to(torch.int32) >> 8) & 0xFF).to(torch.uint8)


# ------------------------------------------------------- level histogram assembly
def assemble_table(slot: np.ndarray, parent: np.ndarray, sib: np.ndarray) -> np.ndarray:
    """hist_assemble's device table: int32 [A, 3] (slot, parent, sibling), flattened."""
    return np.stack([slot, parent, sib], 1).astype(np.int32).reshape(-1)


def hist_assemble(Hb: torch.Tensor, raw_scale, prev: Optional[torch.Tensor], slot: np.ndarray,
                  parent: np.ndarray, sib: np.ndarray, table: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp64 histograms [A, d, B, K] of a level's active nodes in one launch (split.hip): built node a copies
    Hb[slot[a]] (int64 fixed point when ``raw_scale`` is given: a float divides stat 1, a pair (s0, s1)
    divides stats 0 and 1); a derived node (slot -1) is prev[parent[a]] - (its sibling's built histogram).
    ``table``: assemble_table(slot, parent, sib) already on the device (uploaded with the level's other tables)."""
    A = len(slot)
    nb, d, B, Kc = Hb.shape
    dev = Hb.device
    s0, s1 = raw_scales(raw_scale)
    raw = raw_scale is not None
    if not _native(Hb):
        src = Hb.double()
        if raw:
            src = src.clone()
            src[..., 0] /= s0
            src[..., 1] /= s1
        H = torch.empty((A, d, B, Kc), dtype=torch.float64, device=dev)
        sl = torch.from_numpy(np.asarray(slot, dtype=np.int64))
        built = sl >= 0
        if bool(built.any()):
            H[built] = src[sl[built]]
        der = torch.nonzero(~built).flatten()
        if der.numel():
            par = torch.from_numpy(np.asarray(parent, dtype=np.int64))[der]
            sib_ = torch.from_numpy(np.asarray(sib, dtype=np.int64))[der]
            H[der] = prev[par] - src[sl[sib_]]
        return H
    H = torch.empty((A, d, B, Kc), dtype=torch.float64, device=dev)
    m = table if table is not None else upload(dev, assemble_table(slot, parent, sib))[0]
    src = Hb.contiguous() if raw else Hb.double().contiguous()
    if raw:
        assert Hb.dtype == torch.int64
    pv = None if prev is None else prev.contiguous()
    _lib.check(_lib.lib().cdna_hist_assemble(_ptr(src), int(raw), float(s0), float(s1), _ptr(pv),
                                             _ptr(m), A, d * B * Kc, Kc, _ptr(H), _stream(dev)),
               "cdna_hist_assemble")
    return H


def raw_scales(raw_scale):
    """(scale of stat 0, scale of stat 1) of an int64 fixed-point histogram (1.0 = unscaled)."""
    if raw_scale is None:
        return 1.0, 1.0
    if isinstance(raw_scale, (tuple, list)):
        return float(raw_scale[0]), float(raw_scale[1])
    return 1.0, float(raw_scale)


# --------------------------------------------------------------------- K9
GRAD_HESS_OBJ = {"reg:squarederror": 0, "reg:linear": 0, "reg:absoluteerror": 1, "reg:pseudohubererror": 2,
                 "count:poisson": 3, "binary:logistic": 4, "multi:softprob": 5}


def grad_hess(F: torch.Tensor, y: torch.Tensor, w: Optional[torch.Tensor], obj: int):
    """K9: gradient and hessian [n, K] of objective code ``obj`` (GRAD_HESS_OBJ) at margin F [n, K] (GPU).
    y: float labels (class index for softmax); w: optional float row weights.  max |g| is computed in the same
    pass and attached to g as a pending scalar (``prefetch_max``'s attribute: packed_scale_global reads it)."""
    n, Kc = F.shape
    F = F.float().contiguous()
    y = y.float().contiguous()
    w = None if w is None else w.float().contiguous()
    g = torch.empty_like(F)
    h = torch.empty_like(F)
    bits = torch.empty(1, dtype=torch.int32, device=F.device)
    st = torch.cuda.current_stream(F.device)
    _lib.check(_lib.lib().cdna_grad_hess(_ptr(F), _ptr(y), _ptr(w), n, Kc, int(obj), _ptr(g), _ptr(h), _ptr(bits),
                                         st.cuda_stream), "cdna_grad_hess")
    setattr(g, "_cdna_absmax", _PendingScalar(bits.view(torch.float32), st))
    return g, h


# --------------------------------------------------------------------- K3
QUANTILE_MAX_S = 16384  # sample rows a quantile block sorts in LDS (fp64)


def quantile_thresholds(samp: torch.Tensor, max_bins: int):
    """K3 on the GPU: per-feature quantile split candidates of a [s, d] sample in one kernel (quantile.hip).

    Returns host arrays (thr [d, max_bins-1], nthr [d], kdist [d]) and the device tensor of sorted columns
    [d, s] (NaN last), or None when the kernel does not apply (CPU tensor, s > QUANTILE_MAX_S, max_bins < 2).
    Features with kdist <= max_bins (and categorical ones) need the host path on their sorted column."""
    s, d = samp.shape
    if not _native(samp) or s == 0 or s > QUANTILE_MAX_S or not (2 <= max_bins <= 257):
        return None
    samp = samp.double().contiguous()
    dev = samp.device
    sorted_ = torch.empty((d, s), dtype=torch.float64, device=dev)
    thr = torch.empty((d, max_bins - 1), dtype=torch.float64, device=dev)
    ints = torch.empty((2, d), dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().cdna_quantile_thresholds(_ptr(samp), s, d, max_bins, _ptr(sorted_), _ptr(thr),
                                                   _ptr(ints[0]), _ptr(ints[1]), None, _stream(dev)),
               "cdna_quantile_thresholds")
    ih = ints.cpu().numpy()
    return thr.cpu().numpy(), ih[0].copy(), ih[1].copy(), sorted_


class _HostCopies:
    """Device tensors copied to pinned host buffers behind the work already queued; ``get()`` waits for them."""

    def __init__(self, *ts: torch.Tensor):
        self.h = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in ts]
        for hb, t in zip(self.h, ts):
            hb.copy_(t, non_blocking=True)
        self.ev = torch.cuda.Event()
        self.ev.record(torch.cuda.current_stream(ts[0].device))

    def get(self):
        self.ev.synchronize()
        return [hb.numpy() for hb in self.h]


def quantile_thresholds_dev(samp: torch.Tensor, max_bins: int):
    """K3 without a host round trip: (thr [d, max_bins-1] fp32, nthr [d] int32 -- both device tensors, the fp32
    thresholds written by the kernel itself for the binning --, pending host copies of (thr fp64, nthr, kdist)), or
    None where :func:`quantile_thresholds` does not apply.  The binning can be queued on the device thresholds at
    once; they equal the host path's only where every feature has more than ``max_bins`` distinct values (kdist),
    which the caller checks on the host copy once it has queued the binning."""
    s, d = samp.shape
    if not _native(samp) or s == 0 or s > QUANTILE_MAX_S or not (2 <= max_bins <= 257):
        return None
    samp = samp.double().contiguous()
    dev = samp.device
    sorted_ = torch.empty((d, s), dtype=torch.float64, device=dev)
    thr = torch.empty((d, max_bins - 1), dtype=torch.float64, device=dev)
    ints = torch.empty((2, d), dtype=torch.int32, device=dev)
    thr32 = torch.empty((d, max_bins - 1), dtype=torch.float32, device=dev)
    _lib.check(_lib.lib().cdna_quantile_thresholds(_ptr(samp), s, d, max_bins, _ptr(sorted_), _ptr(thr),
                                                   _ptr(ints[0]), _ptr(ints[1]), _ptr(thr32), _stream(dev)),
               "cdna_quantile_thresholds")
    return thr32, ints[0], _HostCopies(thr, ints)


# --------------------------------------------------------------------- K4
# binize v6: the per-feature uniform-grid LUT narrows the threshold search to the few thresholds of the value's cell
# (trees.hip binize5_kernel<C>): cells per feature, 64 or 256; 0 = the 6-step LDS binary search of v5
BINIZE_LUT = 256


def binize(X: torch.Tensor, thr: torch.Tensor, nthr: torch.Tensor, missing: Optional[float] = None,
           want_rm: bool = False, rm_layout: str = "std", out_full=None, row0: int = 0):
    """Raw features -> uint8 bins in feature-group-major layout [G, n, 8].

    want_rm: return ``(bins, rm)`` where ``rm`` is the row-major copy of ``bins_row_major`` written by the
    same kernel (GPU search kernel only; otherwise None and the caller transposes lazily).
    rm_layout "s10" (d <= 100): ``rm`` [n, 16, 8] is in the seg10 layout of :func:`bins_seg10` instead (the
    six-items-per-wave record histogram's rows); None when the kernel that ran cannot write it.

    Continuous feature f: bin = #{thr[f, :nthr[f]] < x}; NaN -> nthr[f].
    Categorical feature (nthr[f] < 0): bin = clamp(int(x), 0, 255).
    missing (XGBoost): values that are NaN or equal ``missing`` are binned as -inf (bin 0 when the
    thresholds start at -FLT_MAX), without materialising a masked copy of X.

    out_full (streamed fits, chunk by chunk): ``(bins [G, N, 8], rm [N, Gs, 8] or None)`` of the whole table;
    this chunk's rows are written to rows [row0, row0 + n) of both, and ``(bins, rm)`` views of them returned.
    """
    n, d = X.shape
    G = (d + 7) // 8
    tmax = thr.shape[1] if thr.dim() == 2 else 0
    if _native(X):
        X = X.float()
        X = X if X.stride(1) == 1 else X.contiguous()
        thr = thr.float().contiguous()
        nthr = nthr.int().contiguous()
        s10 = want_rm and rm_layout == "s10"
        if s10 and d > 100:
            raise ValueError("seg10 rows hold at most 100 features")
        Gs = 16 if (s10 or (BINS_RM_PAD and G <= 16)) else G
        if out_full is not None:
            full, rm_full = out_full
            assert full.shape[0] == G and full.is_contiguous() and row0 + n <= full.shape[1]
            out = full[:, row0:row0 + n]
            ldo, optr = full.shape[1], full.data_ptr() + row0 * 8
            rm = None
            if want_rm:
                assert rm_full is not None and rm_full.shape[1] == Gs and rm_full.is_contiguous()
                rm = rm_full[row0:row0 + n]
        else:
            out = torch.empty((G, n, 8), dtype=torch.uint8, device=X.device)
            ldo, optr = 0, _ptr(out)
            rm = torch.empty((n, Gs, 8), dtype=torch.uint8, device=X.device) if want_rm else None
        miss_on = missing is not None
        miss_val = float("nan") if (missing is None or math.isnan(missing)) else float(missing)
        if n:
            rc = _lib.lib().cdna_binize(_ptr(X), n, d, X.stride(0), _ptr(thr), _ptr(nthr), tmax, int(miss_on),
                                        miss_val, optr, _ptr(rm) if rm is not None else None,
                                        -10 if s10 else Gs, ldo, int(BINIZE_LUT), int(BINIZE_RESIDENT),
                                        _stream(X.device))
            if rc == 2:  # the fallback kernel ran: no row-major copy
                rm = None
            else:
                _lib.check(rc, "cdna_binize")
        return (out, rm) if want_rm else out
    out = torch.zeros((G, n, 8), dtype=torch.uint8) if out_full is None else out_full[0][:, row0:row0 + n]
    if out_full is not None:
        out.zero_()
    Xf = X.float()
    if missing is not None:
        miss = torch.isnan(Xf) if math.isnan(missing) else (torch.isnan(Xf) | (Xf == float(missing)))
        Xf = torch.where(miss, torch.full_like(Xf, float("-inf")), Xf)
    for f in range(d):
        nt = int(nthr[f])
        x = Xf[:, f]
        if nt < 0:
            b = torch.clamp(x.to(torch.int64), 0, 255)
        else:
            b = torch.searchsorted(thr[f, :nt].float().contiguous(), x.contiguous(), right=False)
            b = torch.where(torch.isnan(x), torch.full_like(b, nt), b)
        out[f // 8, :, f % 8] = b.to(torch.uint8)
    return (out, None) if want_rm else out


def bins_seg10(bins: torch.Tensor, d: int) -> torch.Tensor:
    """[G, n, 8] bins -> the seg10 row layout [n, 16, 8] (torch; reference of binize's ``rm_layout="s10"``):
    byte 12 s + p of a row holds feature 10 s + p (s < 10, p < 10), every other byte is 0."""
    G, n, _ = bins.shape
    if d > 100:
        raise ValueError("seg10 rows hold at most 100 features")
    flat = bins.permute(1, 0, 2).reshape(n, G * 8)[:, :d]
    out = torch.zeros((n, 128), dtype=torch.uint8, device=bins.device)
    f = torch.arange(d, device=bins.device)
    out[:, 12 * (f // 10) + f % 10] = flat
    return out.view(n, 16, 8)


def bins_to_matrix(bins: torch.Tensor, d: int) -> torch.Tensor:
    """[G, n, 8] -> [n, d] (int64) view helper for reference code."""
    G, n, _ = bins.shape
    return bins.permute(1, 0, 2).reshape(n, G * 8)[:, :d].to(torch.int64)


# --------------------------------------------------------------------- K5
HIST_LDS_BUDGET = 64 * 1024
# lane mapping: 2 = lane per row (hist4_kernel); 5 = rotated features with the per-update VALU work hoisted
# (hist4f_kernel, when its LDS slot table holds the level's id span)
HIST_MAP = 5
# hist v5 (row records): packed single-atomic regression histograms, trees per block group when packed
HIST5_PACKED = True
HIST5_PACKED_MAXT = 8
HIST5_PACKED_LDS = 128 * 1024
# wave-compacted packed kernel (hist5q): full-wave LDS atomic rounds over sparse (row, tree) work
# 0 off, 1 where it pays (deep levels), 2 always (tests)
HIST5_COMPACT = 1


def _absmax(v: torch.Tensor) -> float:
    """max |v| (NaN if v holds one) in one reduction kernel: the inf-norm reduces |v| inside the reduction, where
    ``v.abs().max()`` first wrote |v| in a full elementwise pass (0.14 ms of a 1e8-row boosting round)."""
    if v.is_floating_point():
        return float(torch.linalg.vector_norm(v.reshape(-1), float("inf")).item())
    return float(v.abs().max().item())


def _fixed_scale(v: Optional[torch.Tensor], n: int, wmax: int, qmax_bits: int = 62) -> float:
    """Power-of-two fixed-point scale so that sum_r w_r * |round(v_r * s)| < 2^62 over n rows
    (and |round(v_r * s)| < 2^qmax_bits for kernels that quantise in 32 bits)."""
    if v is None or v.numel() == 0:
        return 1.0
    m = _absmax(v)
    if not math.isfinite(m):
        raise ValueError("histogram statistic contains NaN/Inf")
    if m == 0.0:
        return 1.0
    e = 62 - math.ceil(math.log2(max(1, n) * max(1, wmax) * m)) - 1
    e = min(e, qmax_bits - math.ceil(math.log2(m)) - 1)
    return float(2.0 ** max(-120, min(100, e)))


# Maxima the host needs before a fit's first level (the label's max |v| for the fixed-point scale, the largest
# bootstrap weight) are reduced on a side stream right after their inputs exist and copied to pinned memory;
# the fit reads them later without draining the device queue (each .item() there idled the GPU ~0.1 ms).
class _PendingScalar:
    def __init__(self, t: torch.Tensor, stream):
        self.host = torch.empty(1, dtype=t.dtype, pin_memory=True)
        self.host.copy_(t.reshape(1), non_blocking=True)
        self.ev = torch.cuda.Event()
        self.ev.record(stream)

    def get(self) -> float:
        self.ev.synchronize()
        return float(self.host[0])


def float_with_absmax(t: torch.Tensor, stream=None) -> torch.Tensor:
    """``t.float()`` of a contiguous fp64 device column with max |t| queued alongside (as prefetch_max(absval)
    attaches it): one pass of misc.hip cast_absmax_kernel instead of cast + abs + max."""
    st = stream if stream is not None else torch.cuda.current_stream(t.device)
    if not (_native(t) and t.dtype == torch.float64 and t.dim() == 1 and t.is_contiguous() and t.numel()):
        with torch.cuda.stream(st):
            out = t.float()
        prefetch_max(out, absval=True, stream=st)
        return out
    with torch.cuda.stream(st):
        out = torch.empty(t.shape, dtype=torch.float32, device=t.device)
        bits = torch.empty(1, dtype=torch.int32, device=t.device)
        rc = _lib.lib().cdna_cast_absmax(_ptr(t), t.numel(), _ptr(out), _ptr(bits), None, st.cuda_stream)
        if rc == 1:  # misaligned view: the torch passes
            out = t.float()
            prefetch_max(out, absval=True, stream=st)
            return out
        _lib.check(rc, "cdna_cast_absmax")
        setattr(out, "_cdna_absmax", _PendingScalar(bits.view(torch.float32), st))
    return out


def shifted_f32(t: torch.Tensor, shift: torch.Tensor) -> torch.Tensor:
    """``(t - shift).float()`` of a contiguous fp64 device column, ``shift`` a one-element fp64 device tensor: one
    pass (misc.hip cast_absmax_kernel with its shift operand), the subtraction in fp64 before the rounding."""
    if not (_native(t) and t.dtype == torch.float64 and t.dim() == 1 and t.is_contiguous() and t.numel()):
        return (t - shift.double()).float()
    sd = shift.double().reshape(1).contiguous()
    out = torch.empty(t.shape, dtype=torch.float32, device=t.device)
    rc = _lib.lib().cdna_cast_absmax(_ptr(t), t.numel(), _ptr(out), None, _ptr(sd), _stream(t.device))
    if rc == 1:  # misaligned view
        return (t - sd).float()
    _lib.check(rc, "cdna_cast_absmax(shift)")
    return out


def sample_rows(n: int, seed: int, offset: int, stream: int, frac: float, device,
                ordered: bool = True) -> Optional[torch.Tensor]:
    """int64 ids of the rows r < n with ``uniform(n, seed, offset, stream)[r] < frac`` (one fused kernel; the set
    of compact_mask(uniform(...) < frac), in arbitrary order unless ``ordered``).  None when the count passes the
    capacity sized from the expected count (the caller then takes the materialised path)."""
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    exp_ = n * frac
    cap = int(exp_ + 12.0 * math.sqrt(exp_ + 1.0) + 1024)
    idx = torch.empty(cap, dtype=torch.int64, device=device)
    cnt = torch.empty(1, dtype=torch.int32, device=device)
    _lib.check(_lib.lib().cdna_sample_rows(n, seed, int(offset), int(stream) & 0xFFFFFFFF, float(frac), _ptr(idx),
                                           cap, _ptr(cnt), _stream(torch.device(device))), "cdna_sample_rows")
    c = int(cnt.item())
    if c > cap:
        return None
    return torch.sort(idx[:c]).values if ordered else idx[:c]


def sample_gather(X: torch.Tensor, seed: int, offset: int, stream: int, frac: float):
    """``X[sample_rows(...)]`` as an fp64 [cap, d] sample without a host round trip: the rows of the Philox sample
    (arbitrary order) then NaN rows up to the capacity (misc.hip sample_gather_kernel).  -> (samp, ok) where
    ``ok()`` (call it once the work behind the sample is queued) tells whether every sampled row fitted the capacity
    (else the caller redoes the exact path); None where the kernels do not apply."""
    n, d = X.shape
    if not _native(X) or n == 0 or X.dtype != torch.float32 or X.stride(1) != 1:
        return None
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    exp_ = n * frac
    cap = int(exp_ + 12.0 * math.sqrt(exp_ + 1.0) + 1024)
    dev = X.device
    idx = torch.empty(8 * cap, dtype=torch.int64, device=dev)  # 8 regions of cap ids (misc.hip)
    cnt = torch.empty(8, dtype=torch.int32, device=dev)
    samp = torch.empty((cap, d), dtype=torch.float64, device=dev)
    _lib.check(_lib.lib().cdna_sample_gather(_ptr(X), n, X.stride(0), d, seed, int(offset) & 0xFFFFFFFFFFFFFFFF,
                                             int(stream) & 0xFFFFFFFF, float(frac), _ptr(idx), _ptr(cnt), cap,
                                             _ptr(samp), _stream(dev)), "cdna_sample_gather")
    host = torch.empty(8, dtype=torch.int32, pin_memory=True)
    host.copy_(cnt, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))

    def ok() -> bool:
        ev.synchronize()
        return int(host.to(torch.int64).sum()) <= cap
    return samp, ok


def prefetch_max(t: torch.Tensor, absval: bool = False, stream=None) -> None:
    """Queue max(t) (max |t|) on ``stream`` (default: current) and attach it to the tensor object itself (never
    keyed by address: a recycled allocation must not inherit a stale value) for packed_scale_global /
    codes_init_max, which then read it instead of syncing."""
    if not t.is_cuda or t.numel() == 0:
        return
    st = stream if stream is not None else torch.cuda.current_stream(t.device)
    with torch.cuda.stream(st):
        m = (t.abs() if absval else t).max()
        setattr(t, "_cdna_absmax" if absval else "_cdna_max", _PendingScalar(m, st))


def _prefetched(t: torch.Tensor, absval: bool) -> Optional[float]:
    p = getattr(t, "_cdna_absmax" if absval else "_cdna_max", None)
    return None if p is None else p.get()


def packed_scale_global(v: torch.Tensor, comm) -> float:
    """``_packed_scale`` from the max |v| over all ranks: every rank quantises identically, so integer
    histograms all-reduce to the same sums whatever the number of GPUs."""
    m = _prefetched(v, True) if v.numel() else 0.0
    if m is None:
        m = _absmax(v)
    m = comm.all_reduce_scalar(m, "max") if comm is not None else m
    if not math.isfinite(m):
        raise ValueError("histogram statistic contains NaN/Inf")
    if m == 0.0:
        return 1.0
    e = math.floor(math.log2((2 ** 23) / m))
    return float(2.0 ** max(-120, min(100, e)))


def _packed_scale(v: torch.Tensor) -> float:
    """Power-of-two scale with |round(v * s)| <= 2^23 (packed count|sum LDS words)."""
    m = _absmax(v) if v.numel() else 0.0
    if not math.isfinite(m):
        raise ValueError("histogram statistic contains NaN/Inf")
    if m == 0.0:
        return 1.0
    e = math.floor(math.log2((2 ** 23) / m))
    return float(2.0 ** max(-120, min(100, e)))


def _hist2(mode: int, bins, d, node, weight, v0, v1, label, C, build_slot, slot_tree, id_tree, feat_mask, B,
           lds_budget, out):
    """Launch the LDS integer histogram kernel (hist4.hip)."""
    S = len(slot_tree)
    G, n, _ = bins.shape
    T = node.shape[0]
    kbits = mode | (4 if (mode == 0 and v0 is not None) else 0)
    per_slot = 8 * B * int(_lib.lib().cdna_hist4_bytes_per_bin(kbits, int(C)))
    SB = max(1, min(S, lds_budget // per_slot))
    if per_slot > 150 * 1024:
        raise ValueError("histogram too large for LDS (classes x bins)")
    slot_tree = np.asarray(slot_tree)
    id_tree = np.asarray(id_tree)
    rows = []
    for a in range(0, S, SB):
        b = min(S, a + SB)
        t0, t1 = int(slot_tree[a]), int(slot_tree[b - 1])
        i0 = int(np.searchsorted(id_tree, t0, side="left"))
        i1 = int(np.searchsorted(id_tree, t1, side="right"))
        rows.append((a, t0, t1, i0, i1))
    grp = torch.tensor(rows, dtype=torch.int32, device=bins.device).reshape(-1)
    ng = len(rows)
    span = max(r[4] - r[3] for r in rows)
    lds_left = 150 * 1024 - ((SB * per_slot + 15) // 16) * 16 - SB - 16
    id_span_max = int(min(span, max(0, lds_left // 4), 16384))
    # 2 x 512-thread blocks per CU when LDS allows; enough chunks to fill 256 CUs
    target = 1024
    nchunk = int(max(1, min((target + G * ng - 1) // (G * ng), (n + 8191) // 8192)))
    nchunk = max(nchunk, -(-n // (1 << 23)))  # u32 LDS counts: rows/chunk * 255 < 2^32
    mw = 0 if feat_mask is None else feat_mask.shape[1]
    fm = None if feat_mask is None else feat_mask.int().contiguous()
    node = node.int().contiguous()
    weight = None if weight is None else weight.to(torch.uint8).contiguous()
    v0 = None if v0 is None else v0.float().contiguous()
    v1 = None if v1 is None else v1.float().contiguous()
    label = None if label is None else label.int().contiguous()
    build_slot = build_slot.int().contiguous()
    vmode = 0
    if HIST_MAP == 5 and v0 is None and id_span_max >= span:
        vmode = 32  # fast rotated kernel (LDS slot table must hold the whole id span)
    wmax = 255 if weight is not None else 1
    qs0 = _fixed_scale(v0, n, wmax)
    qs1 = _fixed_scale(v1, n, wmax, qmax_bits=30 if vmode == 32 else 62)
    iout = torch.zeros(out.shape, dtype=torch.int64, device=bins.device)
    _lib.check(_lib.lib().cdna_hist4(kbits | vmode, _ptr(bins), n, d, T, _ptr(node), _ptr(weight), _ptr(v0),
                                     _ptr(v1), _ptr(label), int(C), _ptr(build_slot), _ptr(fm), mw, S, B, SB,
                                     _ptr(grp), ng, nchunk, id_span_max, qs0, qs1, _ptr(iout),
                                     _stream(bins.device)), "cdna_hist4")
    out.copy_(iout)
    if mode == 0:
        if v0 is not None:
            out[..., 0] /= qs0
        out[..., 1] /= qs1
    return out


def hist_moments(bins: torch.Tensor, d: int, node: torch.Tensor, weight: Optional[torch.Tensor],
                 v0: Optional[torch.Tensor], v1: torch.Tensor, build_slot: torch.Tensor, slot_tree: np.ndarray,
                 feat_mask: Optional[torch.Tensor], B: int, lds_budget: Optional[int] = None,
                 id_tree: Optional[np.ndarray] = None) -> torch.Tensor:
    """Per-slot (feature, bin) weighted moments: out[S, d, B, 2] (float64).

    out[s, f, b, 0] = sum w_t(r) * v0(r), out[s, f, b, 1] = sum w_t(r) * v1(r) over
    rows r whose active node in tree t maps to build slot s and bin_f(r) == b,
    restricted to features enabled in feat_mask[s] (bit f).
    """
    S = len(slot_tree)
    G, n, _ = bins.shape
    T = node.shape[0]
    out = torch.zeros((S, d, B, 2), dtype=torch.float64, device=bins.device)
    if S == 0 or n == 0:
        return out
    if _native(bins):
        assert id_tree is not None, "the GPU node-id histograms need id_tree (the tree of every active node)"
        return _hist2(0, bins, d, node, weight, v0, v1, None, 0, build_slot, slot_tree, id_tree, feat_mask, B,
                      lds_budget or HIST_LDS_BUDGET, out)
    bm = bins_to_matrix(bins, d)
    a0 = torch.ones(n, dtype=torch.float64) if v0 is None else v0.double()
    a1 = v1.double()
    fr = torch.arange(d)
    flat = out.view(-1, 2)
    for t in range(T):
        ids = node[t].long()
        ok = ids >= 0
        slot = torch.full_like(ids, -1)
        slot[ok] = build_slot.long()[ids[ok]]
        ok = slot >= 0
        w = torch.ones(n, dtype=torch.float64) if weight is None else weight[t].double()
        ok = ok & (w != 0)
        if not ok.any():
            continue
        rs = slot[ok]
        idx = (rs[:, None] * d + fr[None, :]) * B + bm[ok]
        msk = torch.ones_like(idx, dtype=torch.bool)
        if feat_mask is not None:
            words = feat_mask.long()[rs]  # [m, MW]
            bits = (words[:, fr // 32] >> (fr % 32)) & 1
            msk = bits.bool()
        wx0 = (w[ok] * a0[ok])[:, None].expand_as(idx)
        wx1 = (w[ok] * a1[ok])[:, None].expand_as(idx)
        flat[:, 0] += torch.bincount(idx[msk], weights=wx0[msk], minlength=flat.shape[0])
        flat[:, 1] += torch.bincount(idx[msk], weights=wx1[msk], minlength=flat.shape[0])
    return out


def hist_classes(bins: torch.Tensor, d: int, node: torch.Tensor, weight: Optional[torch.Tensor],
                 label: torch.Tensor, C: int, build_slot: torch.Tensor, slot_tree: np.ndarray,
                 feat_mask: Optional[torch.Tensor], B: int, lds_budget: Optional[int] = None,
                 id_tree: Optional[np.ndarray] = None) -> torch.Tensor:
    """Per-slot (feature, bin) weighted class counts: out[S, d, B, C] (float64)."""
    S = len(slot_tree)
    G, n, _ = bins.shape
    T = node.shape[0]
    out = torch.zeros((S, d, B, C), dtype=torch.float64, device=bins.device)
    if S == 0 or n == 0:
        return out
    if _native(bins):
        assert id_tree is not None, "the GPU node-id histograms need id_tree (the tree of every active node)"
        return _hist2(1, bins, d, node, weight, None, None, label, C, build_slot, slot_tree, id_tree, feat_mask, B,
                      lds_budget or HIST_LDS_BUDGET, out)
    bm = bins_to_matrix(bins, d)
    lab = label.long()
    fr = torch.arange(d)
    flat = out.view(-1)
    for t in range(T):
        ids = node[t].long()
        ok = ids >= 0
        slot = torch.full_like(ids, -1)
        slot[ok] = build_slot.long()[ids[ok]]
        w = torch.ones(n, dtype=torch.float64) if weight is None else weight[t].double()
        ok = (slot >= 0) & (w != 0) & (lab >= 0) & (lab < C)
        if not ok.any():
            continue
        rs = slot[ok]
        idx = ((rs[:, None] * d + fr[None, :]) * B + bm[ok]) * C + lab[ok][:, None]
        msk = torch.ones_like(idx, dtype=torch.bool)
        if feat_mask is not None:
            words = feat_mask.long()[rs]
            msk = ((words[:, fr // 32] >> (fr % 32)) & 1).bool()
        wx = w[ok][:, None].expand_as(idx)
        flat += torch.bincount(idx[msk], weights=wx[msk], minlength=flat.shape[0])
    return out


# ------------------------------------------------------------ K5/K7 on row records
CODE_DONE = 0xFF


def codes_init(weights: Optional[torch.Tensor], T: int, n: int, device) -> torch.Tensor:
    """Row records for level 0: code[r, t] = weight << 8 | local (0 = the root, 255 = done).

    Returned as int16 [T, n] holding the uint16 bit patterns (hist5.hip)."""
    return codes_init_max(weights, T, n, device)[0]


def codes_init_max(weights: Optional[torch.Tensor], T: int, n: int, device):
    """(codes, largest weight).  On the GPU one kernel writes the codes and reduces the max."""
    if weights is not None and _native(weights) and weights.dtype == torch.uint8 and weights.is_contiguous() \
            and weights.data_ptr() % 16 == 0:
        codes = torch.empty((T, n), dtype=torch.int16, device=weights.device)
        wm = torch.zeros(1, dtype=torch.int32, device=weights.device)
        pre = _prefetched(weights, False)
        _lib.check(_lib.lib().cdna_codes_init(_ptr(weights), T * n, _ptr(codes), _ptr(wm), _stream(weights.device)),
                   "cdna_codes_init")
        return codes, max(1, int(pre if pre is not None else wm.item()))
    if weights is None:
        # every row in every tree with weight 1 at the root (local node 0): one fill, no elementwise chain
        return torch.full((T, n), 1 << 8, dtype=torch.int16, device=device), 1
    else:
        w = weights.to(device=device).to(torch.int32)
    c = (w << 8) | torch.where(w == 0, torch.full_like(w, CODE_DONE), torch.zeros_like(w))
    wmax = int(w.max().item()) if w.numel() else 1
    return c.to(torch.int16).contiguous(), max(1, wmax)


FEATURE_MASKS_MAX_D = 2048


def feature_masks(base: np.ndarray, d: int, k: int, device, base_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-node feature-subset bit words int32 [A, ceil(d/32)] on the GPU (misc.hip feature_masks_kernel): node a
    keeps the k features with the smallest splitmix64(base[a] + f * 0xD6E8FEB86659FD93) -- the words of
    ForestTrainer._feature_masks for the same per-node base.  d <= FEATURE_MASKS_MAX_D."""
    A = len(base)
    W = (d + 31) // 32
    out = torch.empty((A, W), dtype=torch.int32, device=device)
    if A == 0:
        return out
    b = base_dev if base_dev is not None else upload(device, np.ascontiguousarray(base, dtype=np.uint64).view(np.int64))[0]
    _lib.check(_lib.lib().cdna_feature_masks(_ptr(b), A, d, k, _ptr(out), _stream(out.device)), "cdna_feature_masks")
    return out


def decode_codes(codes: torch.Tensor, tfirst: torch.Tensor):
    """codes [T, n] -> (node ids int32 [T, n] with -1 = done, weights uint8 [T, n]).  GPU: one pass
    (seg.hip codes_to_nodes_kernel)."""
    if _native(codes) and codes.dim() == 2 and codes.dtype in (torch.uint16, torch.int16):
        T, n = codes.shape
        c = codes.contiguous()
        tf, = upload(codes.device, tfirst.cpu().numpy().astype(np.int32))
        node = torch.empty((T, n), dtype=torch.int32, device=codes.device)
        w = torch.empty((T, n), dtype=torch.uint8, device=codes.device)
        _lib.check(_lib.lib().cdna_codes_to_nodes(_ptr(c), n, T, _ptr(tf), _ptr(node), _ptr(w), _stream(codes.device)),
                   "cdna_codes_to_nodes")
        return node, w
    c = codes.to(torch.int32) & 0xFFFF
    loc = c & 0xFF
    w = (c >> 8).to(torch.uint8)
    ids = tfirst.to(c.device).to(torch.int32)[:, None] + loc
    ids = torch.where((loc == CODE_DONE) | (w == 0), torch.full_like(ids, -1), ids)
    return ids.contiguous(), w.contiguous()


def hist_codes(mode: int, bins: torch.Tensor, d: int, codes: torch.Tensor, tfirst: torch.Tensor,
               v0: Optional[torch.Tensor], v1: Optional[torch.Tensor], label: Optional[torch.Tensor], C: int,
               build_slot: torch.Tensor, slot_tree: np.ndarray, id_tree: np.ndarray,
               feat_mask: Optional[torch.Tensor], B: int, lds_budget: Optional[int] = None,
               wmax: int = 255) -> torch.Tensor:
    """Histograms from row records (hist5.hip).  mode 0: moments [S, d, B, 2]; 1: classes [S, d, B, C].

    ``wmax``: largest row weight in ``codes`` (bounds the packed kernel's drain interval)."""
    S = len(slot_tree)
    G, n, _ = bins.shape
    T = codes.shape[0] if codes.dim() == 2 else 0
    K_ = 2 if mode == 0 else C
    out = torch.zeros((S, d, B, K_), dtype=torch.float64, device=bins.device)
    if S == 0 or n == 0:
        return out
    if not _native(bins):
        node, w = decode_codes(codes, tfirst)
        if mode == 0:
            return hist_moments(bins, d, node, w, v0, v1, build_slot, slot_tree, feat_mask, B)
        return hist_classes(bins, d, node, w, label, C, build_slot, slot_tree, feat_mask, B)
    lib = _lib.lib()
    maxt = int(lib.cdna_hist5_max_trees())
    packed = HIST5_PACKED and mode == 0 and v0 is None
    compact = packed and HIST5_COMPACT
    kbits = mode | (4 if (mode == 0 and v0 is not None) else 0) | (16 if packed else 0) | (64 if compact else 0)
    per_slot = 8 * B * int(lib.cdna_hist4_bytes_per_bin(kbits, int(C)))
    if per_slot > 150 * 1024:
        raise ValueError("histogram too large for LDS (classes x bins)")
    budget = lds_budget or HIST_LDS_BUDGET
    if packed:
        # register drain holds <= 16 cells per thread: 512 threads -> 64 KB, 1024 threads -> 128 KB
        budget = min(HIST5_PACKED_LDS if lds_budget is None else lds_budget, 16384 * 8)
        maxt = min(maxt, HIST5_PACKED_MAXT)
    SB = max(1, min(S, budget // per_slot))
    slot_tree = np.asarray(slot_tree)
    id_tree = np.asarray(id_tree)
    rows = []
    a = 0
    while a < S:
        b = min(S, a + SB)
        # at most `maxt` trees per group (prefetched row record)
        t0 = int(slot_tree[a])
        b = min(b, int(np.searchsorted(slot_tree, t0 + maxt, side="left")))
        t1 = int(slot_tree[b - 1])
        i0 = int(np.searchsorted(id_tree, t0, side="left"))
        i1 = int(np.searchsorted(id_tree, t1, side="right"))
        rows.append((a, t0, t1, i0, i1))
        a = b
    grp, = upload(bins.device, np.asarray(rows, dtype=np.int32).reshape(-1))
    ng = len(rows)
    # the tree cap can leave groups smaller than the LDS budget allows: size LDS to the largest group
    SB = max(min(SB, (rows[i + 1][0] if i + 1 < ng else S) - rows[i][0]) for i in range(ng))
    max_nt = max(r[2] - r[1] + 1 for r in rows)
    bucket = 1 if max_nt <= 1 else 2 if max_nt <= 2 else 4 if max_nt <= 4 else 8 if max_nt <= 8 else 16
    big = packed and SB * per_slot > 8192 * 8  # 1024-thread blocks: 1 per CU
    # wave compaction pays once the plane needs 1024-thread blocks and several trees share
    # a pass (measured per level: profiles/hist_micro_1e8_compact.txt); below that the
    # lane-per-row kernel's fewer LDS instructions win
    compact = compact and (HIST5_COMPACT >= 2 or (big and max_nt >= 2))
    kbits = kbits if compact else (kbits & ~64)
    rbuf = 16 * 128 * 12 if compact else 0
    lds_used = ((SB * per_slot + 15) // 16) * 16 + rbuf + bucket * 512 + SB + 16
    if lds_used > 160 * 1024:
        raise ValueError("local-node tables do not fit in LDS next to the histogram")
    target_blocks = 512 if big else 1024
    nchunk = int(max(1, min((target_blocks + G * ng - 1) // (G * ng), (n + 8191) // 8192)))
    nchunk = max(nchunk, -(-n // (1 << 23)))
    mw = 0 if feat_mask is None else feat_mask.shape[1]
    fm = None if feat_mask is None else feat_mask.int().contiguous()
    v0 = None if v0 is None else v0.float().contiguous()
    v1 = None if v1 is None else v1.float().contiguous()
    label = None if label is None else label.int().contiguous()
    wmax = int(max(1, min(255, wmax)))
    qs0 = _fixed_scale(v0, n, wmax, qmax_bits=30)
    qs1 = _packed_scale(v1) if packed else _fixed_scale(v1, n, wmax, qmax_bits=30)
    iout = torch.zeros(out.shape, dtype=torch.int64, device=bins.device)
    assert codes.dtype == torch.int16 and codes.is_contiguous() and codes.shape[1] == n
    tf = (upload(bins.device, tfirst.numpy().astype(np.int32))[0] if not tfirst.is_cuda else
          tfirst.to(dtype=torch.int32).contiguous())
    bs = build_slot.int().contiguous()
    _lib.check(lib.cdna_hist5(kbits, _ptr(bins), n, d, T, _ptr(codes), _ptr(tf), _ptr(v0), _ptr(v1), _ptr(label),
                              int(C), _ptr(bs), _ptr(fm), mw, S, B, SB, _ptr(grp), ng, nchunk, max_nt, qs0, qs1,
                              int(max(1, min(255, wmax))), _ptr(iout), _stream(bins.device)), "cdna_hist5")
    out.copy_(iout)
    if mode == 0:
        if v0 is not None:
            out[..., 0] /= qs0
        out[..., 1] /= qs1
    return out


# persistent partition (tables staged once per block, coalesced bins words, all trees' codes in flight)
PARTITION7 = True
PARTITION7_MIN_T = 16



# boosting partitions (partition5 with margins) gather each row's split byte from a feature-major [d][n] byte copy
# of the bins (BinnedData.feature_major_bins, built once per fit) instead of the [G][n] 8-feature words
PART_FEATURE_MAJOR = True


def partition_codes(bins: torch.Tensor, codes: torch.Tensor, tfirst: torch.Tensor, tfirst_next: torch.Tensor,
                    split_feat: torch.Tensor, split_bin: torch.Tensor, cat_off: torch.Tensor,
                    cat_mask: torch.Tensor, child: torch.Tensor, margin: Optional[tuple] = None,
                    bins_fm: Optional[torch.Tensor] = None) -> None:
    """In place: every row's code moves to the chosen child's local index (255 = done).

    margin (GPU, partition5): ``(F [n] fp32, lv [3A] fp32 from split_decode, eta)`` -- rows that finish at this
    level add ``eta * leaf value`` to F (boosting margin update without a tree walk).
    bins_fm (partition5): the feature-major byte copy [G * 8, n] of ``bins`` the row bytes are gathered from."""
    G, n, _ = bins.shape
    T = codes.shape[0]
    if n == 0 or T == 0:
        return
    if _native(bins):
        if not cat_mask.numel():
            cat_mask = torch.zeros(8, dtype=torch.int32)
        srcs = (tfirst, tfirst_next, split_feat, split_bin, cat_off, child, cat_mask)
        if all(not t.is_cuda for t in srcs):
            # one async host->device copy for the seven small tables (seven synchronous copies were ~0.13 ms
            # of launch gaps per level)
            args = upload(bins.device, *[t.numpy().astype(np.int32).reshape(-1) for t in srcs])
        else:
            args = [t.to(device=bins.device, dtype=torch.int32).contiguous() for t in srcs]
        cm = args[6]
        A = int(split_feat.numel())
        # partition7 streams every bins word of every row once per level (10 GB at 1e8 x 100): it pays when
        # many trees share that pass; for few trees partition5's per-(row, tree) byte gathers move less (GBDT,
        # T = 1: 57.9 vs 40.6 ms per boosting round with partition7; CV grid with 5 / 10 trees: 2.18 vs 1.34 s)
        if margin is None and PARTITION7 and T >= PARTITION7_MIN_T and G <= 16 and A <= 1024 and T <= 64:
            _lib.check(_lib.lib().cdna_partition7(
                _ptr(bins), n, G, T, A, _ptr(codes), _ptr(args[0]), _ptr(args[1]), _ptr(args[2]), _ptr(args[3]),
                _ptr(args[4]), _ptr(cm), _ptr(args[5]), _stream(bins.device)), "cdna_partition7")
            return
        F, lv, eta = margin if margin is not None else (None, None, 0.0)
        if margin is not None:
            assert F.dtype == torch.float32 and F.is_contiguous() and F.numel() == n and lv.numel() == 3 * A
        fm = bins_fm is not None
        if fm:
            assert bins_fm.shape == (G * 8, n) and bins_fm.dtype == torch.uint8 and bins_fm.is_contiguous()
        _lib.check(_lib.lib().cdna_partition5(_ptr(bins_fm if fm else bins), n, T, A, _ptr(codes), _ptr(args[0]),
                                              _ptr(args[1]), _ptr(args[2]), _ptr(args[3]), _ptr(args[4]), _ptr(cm),
                                              _ptr(args[5]), -1 if fm else 0, _ptr(lv), float(eta), _ptr(F),
                                              _stream(bins.device)), "cdna_partition5")
        return
    assert margin is None, "margin updates run in the GPU partition only"
    node, w = decode_codes(codes, tfirst)
    live = node >= 0
    partition(bins, node, split_feat, split_bin, cat_off, cat_mask, child)
    tn = tfirst_next.to(torch.int32)[:, None]
    loc = torch.where(node >= 0, node - tn, torch.full_like(node, CODE_DONE))
    loc = torch.where(live, loc, torch.full_like(loc, CODE_DONE))
    c = (w.to(torch.int32) << 8) | loc
    codes.copy_(c.to(torch.int16))


# --------------------------------------------------------------------- K7
def partition(bins: torch.Tensor, node: torch.Tensor, split_feat: torch.Tensor, split_bin: torch.Tensor,
              cat_off: torch.Tensor, cat_mask: torch.Tensor, child: torch.Tensor) -> None:
    """In-place: move each row of each tree from its active node to the chosen child."""
    G, n, _ = bins.shape
    T = node.shape[0]
    if n == 0 or T == 0:
        return
    if _native(bins):
        cm = cat_mask.int().contiguous() if cat_mask.numel() else torch.zeros(8, dtype=torch.int32,
                                                                                 device=bins.device)
        assert node.dtype == torch.int32 and node.is_contiguous()
        split_feat, split_bin = split_feat.int().contiguous(), split_bin.int().contiguous()
        cat_off, child = cat_off.int().contiguous(), child.int().contiguous()
        _lib.check(_lib.lib().cdna_partition(_ptr(bins), n, T, _ptr(node), _ptr(split_feat), _ptr(split_bin),
                                             _ptr(cat_off), _ptr(cm), _ptr(child), _stream(bins.device)),
                   "cdna_partition")
        return
    d = G * 8
    bm = bins_to_matrix(bins, d)
    sf = split_feat.long()
    sb = split_bin.long()
    co = cat_off.long()
    cm = cat_mask.long() & 0xFFFFFFFF
    ch = child.long().view(-1, 2)
    rows = torch.arange(n)
    for t in range(T):
        ids = node[t].long()
        ok = ids >= 0
        if not ok.any():
            continue
        i = ids[ok]
        f = sf[i]
        leaf = f < 0
        fb = bm[rows[ok], f.clamp(min=0)]
        cat = co[i] >= 0
        words = cm[(co[i].clamp(min=0) * 8 + (fb >> 5))] if cm.numel() else torch.zeros_like(fb)
        left = torch.where(cat, ((words >> (fb & 31)) & 1).bool(), fb <= sb[i])
        nxt = torch.where(left, ch[i, 0], ch[i, 1])
        nxt = torch.where(leaf, torch.full_like(nxt, -1), nxt)
        new = ids.clone()
        new[ok] = nxt
        node[t] = new.to(node.dtype)


# --------------------------------------------------------------------- K8
def pack_heap(struct: np.ndarray, vals: np.ndarray, depth: int) -> np.ndarray:
    """Predict-heap table (trees.hip predict_heap_kernel) from a per-slot forest layout.

    ``struct`` int32 [T, 2^(D+1)-1, 2]: per heap slot {feature | -1 leaf/unreachable | -(f+2) categorical,
    threshold bits | mask offset}; ``vals`` float64 [T, 2^(D+1)-1]: the slot's leaf value.  Returns int32
    [T, 2^(D+2)-2]: the 2^D-1 internal slots (leaf slots become pass-through-left), then the 2^D depth-D leaf
    values as fp64, a shallower leaf's value at its leftmost depth-D descendant."""
    T = struct.shape[0]
    NI = (1 << depth) - 1
    out = np.empty((T, 4 * NI + 2), dtype=np.int32)
    out[:, :2 * NI] = struct[:, :NI].reshape(T, 2 * NI)
    leaf = np.zeros((T, NI + 1), dtype=np.float64)
    for k in range(depth, -1, -1):  # shallow last: a reachable leaf overwrites the unreachable slots below it
        s0, s1 = (1 << k) - 1, (1 << (k + 1)) - 1
        tt, ss = np.nonzero(struct[:, s0:s1, 0] == -1)
        if len(tt):
            leaf[tt, (s0 + ss + 1) * (1 << (depth - k)) - 1 - NI] = vals[tt, s0 + ss]
    out[:, 2 * NI:] = leaf.view(np.int32)
    return out


def heap_last_level(so: torch.Tensor, a_tree: torch.Tensor, a_key: torch.Tensor, a_w: torch.Tensor,
                    thr: torch.Tensor, min_gain: float, min_w: float, heap: torch.Tensor, depth: int) -> None:
    """Write a regression forest's last split level into its packed predict heap in place (``pack_heap`` layout
    of depth ``depth``; trees.hip heap_last_level_kernel): for each active node a whose K6 row ``so[a]`` (gain,
    feature, bin, left W, left S, right W, right S, ...) passes the host's split rule (finite gain > 0, >=
    min_gain; node weight a_w[a] >= min_w), the internal slot a_key[a] - 1 gets (feature, fp32 threshold bits of
    thr[feature, bin]) and its two depth-``depth`` leaves S / W (0 for an empty child).  a_tree / a_key int32,
    a_w f64, thr f32 [d, Bt], heap int32 [T, 2^(depth+2)-2]."""
    A = so.shape[0]
    if A == 0:
        return
    T = heap.shape[0]
    NI = (1 << depth) - 1
    assert heap.shape[1] == 4 * NI + 2 and so.dtype == torch.float64
    if _native(so):
        d, Bt = thr.shape
        _lib.check(_lib.lib().cdna_heap_last_level(_ptr(so), so.shape[1], A, _ptr(a_tree), _ptr(a_key), _ptr(a_w),
                                                   _ptr(thr), Bt, d, float(min_gain), float(min_w), _ptr(heap),
                                                   depth, T, _stream(so.device)), "cdna_heap_last_level")
        return
    gain = so[:, 0]
    ok = torch.isfinite(gain) & (gain > 0) & (gain >= min_gain) & (a_w >= min_w)
    idx = torch.nonzero(ok).flatten()
    if not len(idx):
        return
    f, b = so[idx, 1].long(), so[idx, 2].long()
    t, k = a_tree[idx].long(), a_key[idx].long()
    heap[t, 2 * (k - 1)] = f.to(torch.int32)
    heap[t, 2 * (k - 1) + 1] = thr[f, b].float().view(torch.int32)
    leaf = heap[:, 2 * NI:].view(torch.float64)  # [T, 2^depth] (a view: writes land in heap)
    for side in (0, 1):
        W, S = so[idx, 3 + 2 * side], so[idx, 4 + 2 * side]
        leaf[t, 2 * k + side - (1 << depth)] = torch.where(W > 0, S / torch.where(W > 0, W, torch.ones_like(W)),
                                                           torch.zeros_like(W))


def ordered_tree_sum(contribs, T: int, n: int, K: int, base=None) -> torch.Tensor:
    """The fp64 ensemble sum in the device kernels' order (trees.hip predict_kernel): lane q = t % 4 adds
    ``contribs(t)`` (tree_w[t] * leaf value, already a rounded product) for its trees in ascending order, then
    base + lane 0 + lane 1 + lane 2 + lane 3.  The cpu predictions therefore equal the GPU's bit for bit."""
    lanes = [torch.zeros((n, K), dtype=torch.float64) for _ in range(4)]
    for t in range(T):
        lanes[t & 3] += contribs(t)
    out = torch.zeros((n, K), dtype=torch.float64)
    if base is not None:
        out += base.double().cpu()[None, :]
    for q in range(4):
        out += lanes[q]
    return out


# persistent one-round grids (exactly the resident blocks) for the streaming kernels -- binize v5 and the heap
# predict -- instead of fixed caps of 1024 / 8192 blocks (per-block setup and the uneven last trips are what made
# them 8-9 % slower per row at the 8-GPU shard size: VERDICT r5 weak #2)
# (A/B round 6, profiles/r6/headline_ab.md: one persistent round was 0.4 ms SLOWER at the headline and within noise
# at the 8-GPU shard size, so both stay off)
BINIZE_RESIDENT = False
PREDICT_RESIDENT = False


def tree_predict_heap(X: torch.Tensor, heap: torch.Tensor, depth: int, tree_w: torch.Tensor,
                      masks: torch.Tensor, base: float = 0.0, dtype=torch.float64) -> Optional[torch.Tensor]:
    """Single-output ensemble prediction over a packed heap forest (int32 [T, 2^(depth+2)-2], ``pack_heap``):
    fp64 leaves, weights and sums (Spark's Double predictions), stored as ``dtype``.  Returns None when the forest
    does not fit the kernel's LDS budget (use ``tree_predict``)."""
    n, d = X.shape
    T = heap.shape[0]
    if not _native(X):
        return None
    assert heap.dtype == torch.int32 and heap.dim() == 2 and heap.shape[1] == (4 << depth) - 2, \
        (tuple(heap.shape), depth)
    X = X.float()
    X = X if X.stride(1) == 1 else X.contiguous()
    out = torch.empty((n, 1), dtype=dtype, device=X.device)
    if n == 0:
        return out
    m = masks.int().contiguous() if masks.numel() else torch.zeros(8, dtype=torch.int32, device=X.device)
    f64 = dtype == torch.float64
    assert tree_w.numel() == T
    rc = _lib.lib().cdna_tree_predict_heap(_ptr(X), n, d, X.stride(0), _ptr(heap.contiguous()), depth,
                                           _ptr(tree_w.double().contiguous()), T, _ptr(m), float(base),
                                           None if f64 else _ptr(out), _ptr(out) if f64 else None,
                                           int(PREDICT_RESIDENT), _stream(X.device))
    if rc == 1:  # hipErrorInvalidValue: over the LDS budget
        return None
    _lib.check(rc, "cdna_tree_predict_heap")
    return out


def bin_upper_edges(thresholds: np.ndarray, nthr: np.ndarray, B: int) -> np.ndarray:
    """[d, B] fp32: feature f's bin b -> the fp32 threshold t_b the bins were cut with (binize: bin(x) = #{t_j <
    x}), +inf for b >= nthr[f] (the last bin and NaN).  ``tree_predict_heap_binned``'s dequantisation table."""
    d = thresholds.shape[0]
    up = np.full((d, B), np.inf, dtype=np.float32)
    for f in range(d):
        k = int(min(max(nthr[f], 0), B, thresholds.shape[1]))
        up[f, :k] = thresholds[f, :k].astype(np.float32)
    return up


def heap_predict_host(Xf: torch.Tensor, heap: torch.Tensor, depth: int, tree_w: torch.Tensor,
                      base: float = 0.0) -> torch.Tensor:
    """Host walk of a packed predict heap (numeric and pass-through slots) on fp32 rows -> [n] fp64, summed in the
    device kernels' order (``ordered_tree_sum``): the cpu twin of ``tree_predict_heap`` and, on dequantised bins
    (``bin_upper_edges``), of ``tree_predict_heap_binned``."""
    Xf = Xf.float().cpu()
    h = heap.cpu()
    n, T = Xf.shape[0], h.shape[0]
    NI = (1 << depth) - 1
    tw = tree_w.double().cpu()
    rows = torch.arange(n)

    def contrib(t):
        slots = h[t, :2 * NI].reshape(max(NI, 0), 2)
        leaf = h[t, 2 * NI:].contiguous().view(torch.float64)
        idx = torch.zeros(n, dtype=torch.long)
        for _ in range(depth):
            nd = slots[idx]
            f = nd[:, 0].long()
            if bool((f < -1).any()):
                raise ValueError("heap_predict_host: categorical slots are not supported")
            thr = nd[:, 1].contiguous().view(torch.float32)
            x = Xf[rows, f.clamp(min=0)]
            go_left = (f < 0) | (x <= thr)
            idx = 2 * idx + torch.where(go_left, 1, 2)
        return (tw[t] * leaf[idx - NI])[:, None]
    out = ordered_tree_sum(contrib, T, n, 1, torch.tensor([float(base)], dtype=torch.float64))
    return out[:, 0]


def tree_predict_heap_binned(bins: torch.Tensor, thr_up: torch.Tensor, d: int, heap: torch.Tensor, depth: int,
                             tree_w: torch.Tensor, base: float = 0.0, dtype=torch.float64) -> Optional[torch.Tensor]:
    """``tree_predict_heap`` over the uint8 bins the features were cut into (trees.hip predict_heap_binned_kernel):
    bins [G, n, 8] (binize's column groups), thr_up fp32 [d, B] (``bin_upper_edges``).  x <= v <=> t_bin(x) <= v
    for every threshold v of the binning, so the predictions equal ``tree_predict_heap`` on the fp32 rows bit for
    bit.  [n, 1] ``dtype``; None when over the kernel's LDS budget.  Numeric / pass-through heap slots only."""
    G, n, _ = bins.shape
    T = heap.shape[0]
    assert heap.dtype == torch.int32 and heap.dim() == 2 and heap.shape[1] == (4 << depth) - 2, \
        (tuple(heap.shape), depth)
    assert thr_up.dtype == torch.float32 and thr_up.dim() == 2 and thr_up.shape[0] == d and d <= 8 * G
    assert tree_w.numel() == T
    if not _native(bins):
        b = bins_to_matrix(bins, d).cpu().clamp(max=thr_up.shape[1] - 1)
        Xq = thr_up.cpu().gather(1, b.t().contiguous()).t()   # [n, d]: each bin's upper edge
        return heap_predict_host(Xq, heap, depth, tree_w, base).to(dtype)[:, None].to(bins.device)
    out = torch.empty((n, 1), dtype=dtype, device=bins.device)
    if n == 0:
        return out
    f64 = dtype == torch.float64
    heap = heap.contiguous()
    heap_b = torch.empty_like(heap)  # the slots as bin counts (trees.hip heap_to_bins_kernel)
    rc = _lib.lib().cdna_tree_predict_heap_binned(_ptr(bins.contiguous()), n, G, d, _ptr(thr_up.contiguous()),
                                                  thr_up.shape[1], _ptr(heap), depth,
                                                  _ptr(tree_w.double().contiguous()), T, float(base), _ptr(heap_b),
                                                  None if f64 else _ptr(out), _ptr(out) if f64 else None,
                                                  _stream(bins.device))
    if rc == 1:
        return None
    _lib.check(rc, "cdna_tree_predict_heap_binned")
    return out


def tree_predict(X: torch.Tensor, nodes: torch.Tensor, roots: torch.Tensor, tree_w: torch.Tensor,
                 values: torch.Tensor, masks: torch.Tensor, K: int, base: Optional[torch.Tensor] = None
                 ) -> torch.Tensor:
    """Ensemble prediction on raw features -> float64 [n, K] (fp64 leaf values, weights and sums; the cpu path
    sums in the kernel's order: ``ordered_tree_sum``).

    nodes: int32 [N, 4] packed as documented in trees.hip.
    """
    n, d = X.shape
    T = roots.numel()
    if _native(X):
        X = X.float()
        X = X if X.stride(1) == 1 else X.contiguous()
        out = torch.empty((n, K), dtype=torch.float64, device=X.device)
        if n:
            m = masks.int().contiguous() if masks.numel() else torch.zeros(8, dtype=torch.int32, device=X.device)
            nodes, roots = nodes.int().contiguous(), roots.int().contiguous()
            tree_w, values = tree_w.double().contiguous(), values.double().contiguous()
            base = None if base is None else base.double().contiguous()
            _lib.check(_lib.lib().cdna_tree_predict(_ptr(X), n, d, X.stride(0), _ptr(nodes), int(nodes.shape[0]),
                                                    _ptr(roots),
                                                    _ptr(tree_w), T, _ptr(values), _ptr(m), K, _ptr(base), _ptr(out),
                                                    int(values.numel()), _stream(X.device)), "cdna_tree_predict")
        return out
    Xf = X.float().cpu()
    nd = nodes.long().cpu()
    vals = values.double().cpu()
    tw = tree_w.double().cpu()
    mk = masks.long().cpu() & 0xFFFFFFFF
    rows = torch.arange(n)

    def contrib(t):
        cur = torch.full((n,), int(roots[t]), dtype=torch.long)
        for _ in range(64):
            nv = nd[cur]
            internal = nv[:, 0] != -1
            if not internal.any():
                break
            f = nv[:, 0]
            cont = f >= 0
            fi = torch.where(cont, f, -f - 2).clamp(min=0)
            x = Xf[rows, fi]
            thr = nv[:, 1].to(torch.int32).view(torch.float32)
            c = x.to(torch.int64)
            okc = (c >= 0) & (c < 256)
            cc = c.clamp(0, 255)
            moff = torch.where(f <= -2, nv[:, 1], torch.zeros_like(f)).clamp(min=0)
            words = mk[(moff * 8 + (cc >> 5))] if mk.numel() else torch.zeros_like(cc)
            catleft = okc & ((words >> (cc & 31)) & 1).bool()
            left = torch.where(cont, x <= thr, catleft)
            nxt = torch.where(left, nv[:, 2], nv[:, 3])
            cur = torch.where(internal, nxt, cur)
        off = nd[cur][:, 1]
        idx = off[:, None] + torch.arange(K)[None, :]
        return vals[idx] * tw[t]
    return ordered_tree_sum(contrib, T, n, K, base).to(X.device)


def predict_binned_add(bins: torch.Tensor, nodes: torch.Tensor, root: int, values: torch.Tensor,
                       masks: torch.Tensor, scale: float, out: torch.Tensor) -> None:
    """out[r] += scale * leaf value of a bin-threshold tree (GBDT margin update).

    (A/B, profiles/r4/gbdt_predict_ab.md: the tree in LDS with four walks per thread measured 3.16 ms and a
    row-major walk 14 ms against this kernel's 2.37 ms per round at 1e8 rows; both dropped.)"""
    G, n, _ = bins.shape
    if n == 0:
        return
    if _native(bins):
        m = masks.int().contiguous() if masks.numel() else torch.zeros(8, dtype=torch.int32, device=bins.device)
        nodes, values = nodes.int().contiguous(), values.float().contiguous()
        assert out.dtype == torch.float32 and out.is_contiguous()
        _lib.check(_lib.lib().cdna_predict_binned_add(_ptr(bins), n, _ptr(nodes), int(root), _ptr(values), _ptr(m),
                                                      float(scale), _ptr(out), _stream(bins.device)),
                   "cdna_predict_binned_add")
        return
    bm = bins_to_matrix(bins, G * 8)
    nd = nodes.long()
    mk = masks.long() & 0xFFFFFFFF
    rows = torch.arange(n)
    cur = torch.full((n,), int(root), dtype=torch.long)
    for _ in range(64):
        nv = nd[cur]
        internal = nv[:, 0] != -1
        if not internal.any():
            break
        f = nv[:, 0]
        cont = f >= 0
        fi = torch.where(cont, f, -f - 2).clamp(min=0)
        b = bm[rows, fi]
        moff = torch.where(f <= -2, nv[:, 1], torch.zeros_like(f)).clamp(min=0)
        words = mk[(moff * 8 + (b >> 5))] if mk.numel() else torch.zeros_like(b)
        left = torch.where(cont, b <= nv[:, 1], ((words >> (b & 31)) & 1).bool())
        cur = torch.where(internal, torch.where(left, nv[:, 2], nv[:, 3]), cur)
    out += scale * values.float()[nd[cur][:, 1]]


def predict_binned_forest_host(bins: torch.Tensor, trees, scale: float, F: torch.Tensor) -> None:
    """Host twin of ``predict_binned_add`` over a WHOLE forest: every tree walks at once (one [T*n] cursor),
    so a 100-tree margin costs ~depth vector steps instead of 100 x depth.  ``trees[t] = (nodes, values,
    masks)`` as ``Forest.binned_arrays``; tree t adds to column ``t % F.shape[1]``, summed tree by tree in
    float32 like the per-tree path (identical results)."""
    G, n, _ = bins.shape
    T = len(trees)
    if n == 0 or T == 0:
        return
    bm = bins_to_matrix(bins, G * 8)
    nodes, vals, masks, roots = [], [], [], []
    no = vo = mo = 0
    for nd_t, v_t, m_t in trees:
        nd_t = nd_t.long().clone()
        leaf = nd_t[:, 0] == -1
        cat = nd_t[:, 0] <= -2
        nd_t[~leaf, 2:] += no
        nd_t[leaf, 1] += vo
        nd_t[cat, 1] += mo
        roots.append(no)
        nodes.append(nd_t)
        vals.append(v_t.float().reshape(-1))
        m_t = m_t.long().reshape(-1) & 0xFFFFFFFF
        masks.append(m_t)
        no += nd_t.shape[0]
        vo += vals[-1].numel()
        mo += m_t.numel() // 8
    nd = torch.cat(nodes)
    mk = torch.cat(masks)
    vv = torch.cat(vals)
    rows = torch.arange(n).repeat(T)
    cur = torch.tensor(roots, dtype=torch.long).repeat_interleave(n)
    for _ in range(64):
        nv = nd[cur]
        internal = nv[:, 0] != -1
        if not internal.any():
            break
        f = nv[:, 0]
        cont = f >= 0
        fi = torch.where(cont, f, -f - 2).clamp(min=0)
        b = bm[rows, fi]
        moff = torch.where(f <= -2, nv[:, 1], torch.zeros_like(f)).clamp(min=0)
        words = mk[(moff * 8 + (b >> 5))]
        left = torch.where(cont, b <= nv[:, 1], ((words >> (b & 31)) & 1).bool())
        cur = torch.where(internal, torch.where(left, nv[:, 2], nv[:, 3]), cur)
    leafv = vv[nd[cur][:, 1]].view(T, n)
    K = F.shape[1]
    for t in range(T):
        F[:, t % K] += scale * leafv[t]


# -------------------------------------------------------------------- K13
def reg_metrics(y: torch.Tensor, p: torch.Tensor, w: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[Σw, Σw e², Σw|e|, Σw y, Σw y², Σw p, Σw p², Σw y p] as float64[8] (local)."""
    y = y.double().contiguous()
    p = p.double().contiguous()
    w = None if w is None else w.double().contiguous()
    if _native(y):
        acc = torch.zeros(8, dtype=torch.float64, device=y.device)
        part = torch.empty(8 * 1024, dtype=torch.float64, device=y.device)  # per-block partials (fixed-order sum)
        _lib.check(_lib.lib().cdna_reg_metrics(_ptr(y), _ptr(p), _ptr(w), y.numel(), _ptr(part), _ptr(acc),
                                               _stream(y.device)), "cdna_reg_metrics")
        return acc
    ww = torch.ones_like(y) if w is None else w
    e = y - p
    return torch.stack([ww.sum(), (ww * e * e).sum(), (ww * e.abs()).sum(), (ww * y).sum(), (ww * y * y).sum(),
                        (ww * p).sum(), (ww * p * p).sum(), (ww * y * p).sum()])


# -------------------------------------------------------------------- K14
def score_hist(score: torch.Tensor, label: torch.Tensor, lo: float, hi: float, nb: int) -> torch.Tensor:
    score = score.double().contiguous()
    label = label.double().contiguous()
    if _native(score):
        h = torch.zeros((nb, 2), dtype=torch.float64, device=score.device)
        _lib.check(_lib.lib().cdna_score_hist(_ptr(score), _ptr(label), score.numel(), float(lo), float(hi), nb,
                                              _ptr(h), _stream(score.device)), "cdna_score_hist")
        return h
    scale = nb / (hi - lo) if hi > lo else 0.0
    b = ((score - lo) * scale).floor().long().clamp(0, nb - 1)
    pos = (label > 0.5).long()
    h = torch.zeros(nb * 2, dtype=torch.float64)
    h.index_add_(0, b * 2 + pos, torch.ones_like(score))
    return h.view(nb, 2)


# -------------------------------------------------------------------- K10
def kmeans_step(X: torch.Tensor, C: torch.Tensor, with_sums: bool = True):
    """Assign rows to nearest centre; return (assign, sums[k,d], counts[k], cost) (local)."""
    n, d = X.shape
    k = C.shape[0]
    f64 = X.dtype == torch.float64   # Spark's Double vectors at course scale: the fp64 kernel instantiation
    if _native(X) and (2 * k * d + k) * (8 if f64 else 4) <= 64 * 1024:
        X = X if f64 else X.float()
        X = X if X.stride(1) == 1 else X.contiguous()
        Cf = C.to(X.dtype).contiguous()
        assign = torch.empty(n, dtype=torch.int32, device=X.device)
        sums = torch.zeros((k, d), dtype=torch.float64, device=X.device)
        counts = torch.zeros(k, dtype=torch.float64, device=X.device)
        cost = torch.zeros(1, dtype=torch.float64, device=X.device)
        if n:
            _lib.check(_lib.lib().cdna_kmeans_step(_ptr(X), n, d, X.stride(0), _ptr(Cf), k, _ptr(assign),
                                                   _ptr(sums) if with_sums else None,
                                                   _ptr(counts) if with_sums else None, _ptr(cost), int(f64),
                                                   _stream(X.device)), "cdna_kmeans_step")
        return assign, sums, counts, cost[0]
    Xf = X if f64 else X.float()
    dist = ((Xf[:, None, :] - C.to(Xf.dtype)[None, :, :]) ** 2).sum(2) if f64 else torch.cdist(Xf, C.float()) ** 2
    best, assign = dist.min(dim=1)
    sums = torch.zeros((k, d), dtype=torch.float64, device=X.device)
    sums.index_add_(0, assign, Xf.double())
    counts = torch.bincount(assign, minlength=k).double()
    return assign.int(), sums, counts, best.double().sum()


# -------------------------------------------------------------------- K11
def logistic_grad(X: torch.Tensor, y: torch.Tensor, w: torch.Tensor, b: float,
                  wt: Optional[torch.Tensor] = None):
    """Binary logistic loss and gradient (local sums): returns (grad[d+1], loss)."""
    n, d = X.shape
    y = y.double().contiguous()
    wt = None if wt is None else wt.double().contiguous()
    if _native(X) and d <= 512:
        f64 = X.dtype == torch.float64   # Double vectors (course scale): the fp64 instantiation reads them as is
        X = X if f64 else X.float()
        X = X if X.stride(1) == 1 else X.contiguous()
        wd = w.double().contiguous()
        grad = torch.zeros(d + 1, dtype=torch.float64, device=X.device)
        loss = torch.zeros(1, dtype=torch.float64, device=X.device)
        if n:
            _lib.check(_lib.lib().cdna_logistic_grad(_ptr(X), n, d, X.stride(0), _ptr(y), _ptr(wt), _ptr(wd),
                                                     float(b), _ptr(grad), _ptr(loss), int(f64), _stream(X.device)),
                       "cdna_logistic_grad")
        return grad, loss[0]
    Xd = X.double()
    m = Xd @ w.double() + b
    p = torch.sigmoid(m)
    ww = torch.ones_like(y) if wt is None else wt
    res = ww * (p - y)
    g = torch.empty(d + 1, dtype=torch.float64, device=X.device)
    g[:d] = Xd.T @ res
    g[d] = res.sum()
    loss = (ww * (torch.nn.functional.softplus(m) - y * m)).sum()
    return g, loss


# ------------------------------------------------------------ segment mode (seg.hip)
SEG_HIST_CHUNK = 262144
# lane10 record chunks (levels 2-4 of the headline): at most this many records per block.  The records of a slot
# are in row order and the work list interleaves the slots by relative position, so smaller chunks keep the ~256
# concurrently running blocks on a narrower row window (each row line is gathered by ~6.3 slots at the headline:
# scripts/level_records.py); 16384 blocks per level measured -0.7 ms at 1e8 rows, and the per-rank shape keeps its
# ~37K-record chunks (SEG_MIN_BLOCKS) -- profiles/r6/headline_ab.md
LANE10_CHUNK_MAX = 40960
# row-major bins copy for segment histograms (one cache line per row instead of one per 8-feature group)
SEG_ROW_MAJOR = True
SEG_PART_CHUNK = 8192


def seg_scales(v0p: Optional[torch.Tensor], v1p: torch.Tensor, wmax: int, n_global: int, comm=None):
    """Fixed-point scales for one tree's statistics (packed when there is no v0).

    With ``comm`` the max |v|, the max weight and ``n_global`` are agreed over every rank first: all ranks
    then quantise identically and their int64 histograms all-reduce to the same sums on 1 or N GPUs."""
    if v0p is None:
        return 1.0, (packed_scale_global(v1p, comm) if comm is not None else _packed_scale(v1p))
    if comm is None or not comm.distributed:
        return (_fixed_scale(v0p, n_global, wmax, qmax_bits=30), _fixed_scale(v1p, n_global, wmax, qmax_bits=30))
    m = torch.tensor([_absmax(v0p) if v0p.numel() else 0.0,
                      _absmax(v1p) if v1p.numel() else 0.0, float(wmax)], dtype=torch.float64)
    comm.all_reduce(m, "max")
    w = int(m[2])
    return (_fixed_scale(m[0:1], n_global, w, qmax_bits=30), _fixed_scale(m[1:2], n_global, w, qmax_bits=30))


SEG_MIN_BLOCKS = 2048
SEG_ROUND_FIT = True
# wide-bin (80 < B <= 256, boosting) record levels: work items per level (x ceil(d / 64) feature blocks).  Every block
# clears and flushes 64 features x B bins of LDS cells into the level histogram with global atomics, so at deep
# boosting levels (fewer rows, the same number of blocks) the flush -- not the rows -- sets the level time.
# bench_configs.py gbdt (1e8 x 100, 256 bins), 3 interleaved reps: 1024 -> 28.05-28.23, 768 -> 27.83-27.85,
# 512 -> 27.78-27.83 ms per tree (profiles/r4/gbdt_min_blocks_ab.txt)
SEG_MIN_BLOCKS_WIDE = 512
# three-times-larger record chunks for the six-items-per-wave kernel (its count field is spread over three cell
# copies): measured 145.1 vs 139.8 ms per headline step (fewer, longer blocks) and neutral at 1.25e7 rows -- off
LANE10_CHUNK3 = False
# record histograms through the lane-feature kernel (seg_hist_lane_kernel: lanes own features, bin-major
# conflict-free LDS planes, one v_perm per cell address); B <= 80 (4 planes <= 80 KB of LDS), 80 < B <= 256:
# seg_hist_lane4_kernel (64 features per block, a quarter-wave per item; SEG_LANE=False keeps the flat kernel)
SEG_LANE = True
# seg10 rows + the six-items-per-wave record histogram for 80 < d <= 100, B <= 40 (SEG10=False: lane8 rows)
SEG10 = True
SEG_LANE_MAX_B = 256
# records buffers carry REC_PAD readable entries past their end: the lane kernel's record loads are unconditional
REC_PAD = 128


# the record histograms' host planning (_fill_chunk + _seg_work) in the native library (csrc/kernels/plan.hip): ~250 us
# of numpy per level -> a few us, off the GPU's critical path at the 8-GPU shard size
NATIVE_PLAN = True


def _seg_plan(segs: np.ndarray, chunk: int, B: int, ncu: int, interleave: bool):
    """(chunk, work) = (_fill_chunk(segs, chunk, B, ncu), _seg_work(segs, that chunk, interleave)), natively."""
    segs = np.ascontiguousarray(np.asarray(segs, dtype=np.int64).reshape(-1, 3))
    k = len(segs)
    mb = SEG_MIN_BLOCKS if B <= 64 else min(SEG_MIN_BLOCKS, SEG_MIN_BLOCKS_WIDE)
    L = _lib.lib()
    lens = np.ascontiguousarray(segs[:, 1])
    c = int(L.cdna_fill_chunk(lens.ctypes.data, k, int(chunk), int(B), int(ncu), int(mb)))
    total = int(lens.clip(min=0).sum())
    cap = total // max(1, c) + k + 1
    out = np.empty((cap, 3), dtype=np.int32)
    m = int(L.cdna_seg_work(segs.ctypes.data, k, c, int(bool(interleave)), out.ctypes.data, cap))
    assert m >= 0, (m, cap)
    return c, out[:m]


def _fill_chunk(segs: np.ndarray, chunk: int, B: int = 0, ncu: int = 0) -> int:
    """Shrink the rows-per-block chunk so a level with few rows still launches ~SEG_MIN_BLOCKS blocks
    (at 1.25e7 rows per GPU a level's 95K-row chunks made only ~100 blocks for 256 CUs).  With 2048 instead of
    1024 the per-rank shape of the 8-GPU point ran 22.6 -> 21.2 ms (the last round of blocks no longer idles
    half the chip); wide-bin levels (B > 64: 128 KB LDS planes to clear and flush per block) keep 1024.

    ncu > 0 (one block per CU, B <= 64): when the per-segment rounding leaves a last round of blocks less than
    half full (2048 target blocks + one partial chunk per segment = 8 rounds + a sliver), the chunk grows -- up to
    ``chunk`` -- just enough for the blocks to fit the whole rounds before it."""
    lens = np.asarray(segs, dtype=np.int64).reshape(-1, 3)[:, 1].clip(min=0)
    total = int(lens.sum())
    mb = SEG_MIN_BLOCKS if B <= 64 else min(SEG_MIN_BLOCKS, SEG_MIN_BLOCKS_WIDE)
    c0 = int(min(chunk, max(8192, -(-total // max(1, mb)))))
    if ncu <= 0 or B > 64 or c0 >= chunk:
        return c0
    lens = lens[lens > 0]
    blocks = int(((lens + c0 - 1) // c0).sum())
    R, rem = divmod(blocks, ncu)
    if R < 1 or rem == 0 or rem > ncu // 2:
        return c0
    lo, hi = c0, int(chunk)
    if int(((lens + hi - 1) // hi).sum()) > R * ncu:
        return c0
    # the answer c satisfies total / c <= sum ceil(len / c) <= R * ncu and sum ceil(len / c) <= total / c + k:
    # it lies in [total / (R ncu), total / (R ncu - k)] (a few bisection steps, not ~17 over [c0, chunk])
    cap = R * ncu
    lo = max(lo, -(-total // cap))
    if cap > len(lens):
        hi = min(hi, -(-total // (cap - len(lens))))
    while lo < hi:  # smallest chunk whose blocks fit R rounds
        mid = (lo + hi) // 2
        if int(((lens + mid - 1) // mid).sum()) <= R * ncu:
            hi = mid
        else:
            lo = mid + 1
    return lo


def _seg_work(segs: np.ndarray, chunk: int, interleave: bool = False) -> np.ndarray:
    """segs [k, 3] {start, len, tag} -> work items [m, 3] of at most `chunk` rows each.

    interleave: ordered by relative position inside the segment, so that concurrently running blocks gather nearby
    rows (chunk j of every segment covers about the same fraction of the row ids; placing rounds of chunks on one
    XCD for L2 sharing measured no better and was dropped), built in the same pass: the
    position is bucketed to a uint16 key (chunk j of a k-chunk segment -> j * kmax // k), whose stable argsort is a
    radix sort -- the float key's merge sort plus a second pass cost ~60-70 us of host time per level at the
    per-rank shape, while the GPU waited.  Any order gives the same histograms (exact fixed-point sums)."""
    segs = np.asarray(segs, dtype=np.int64).reshape(-1, 3)
    segs = segs[segs[:, 1] > 0]
    if len(segs) == 0:
        return np.zeros((0, 3), dtype=np.int32)
    k = (segs[:, 1] + chunk - 1) // chunk
    rep = np.repeat(np.arange(len(segs)), k)
    j = np.arange(len(rep)) - (np.cumsum(k) - k)[rep]
    if interleave and len(segs) > 1:
        kmax = int(k.max())
        key = j * kmax // k[rep]
        if kmax < 1 << 16:
            key = key.astype(np.uint16)
        o = np.argsort(key, kind="stable")
        rep, j = rep[o], j[o]
    out = np.empty((len(rep), 3), dtype=np.int32)
    out[:, 0] = segs[rep, 0] + j * chunk
    out[:, 1] = np.minimum(chunk, segs[rep, 1] - j * chunk)
    out[:, 2] = segs[rep, 2]
    return out


def seg_hist(bins: torch.Tensor, d: int, B: int, perm: torch.Tensor, v0p: Optional[torch.Tensor],
             v1p: torch.Tensor, wp: Optional[torch.Tensor], segs: np.ndarray, S: int, wmax: int,
             scales=None, bins_rm: Optional[torch.Tensor] = None, interleave: bool = False,
             rec: bool = False, raw: bool = False, out: Optional[torch.Tensor] = None,
             rm_s10: bool = False, cls3: bool = False) -> torch.Tensor:
    """Moments [S, d, B, 2] of node segments of ``perm`` (row ids grouped by node).

    rm_s10 (rec): ``bins_rm`` is in the seg10 layout (:func:`bins_seg10`): the six-items-per-wave kernel.

    cls3 (rec + raw): 3-class records (label codes 0 / 1 / ``CLS3_CODE``, scale 1): the sums are [S, d, B, 3]
    (W, W1, W2) (:func:`cls3_expand` turns them into class counts).

    out (rec + raw): a zeroed int64 [S, d, B, 2] tensor (e.g. a slot-range slice of a level's buffer) the sums
    are accumulated into and returned -- lets the engine all-reduce one slot chunk while the next is built.

    rec: ``perm`` holds packed int64 item records from ``codes_compact(rec_scale=scales[1])`` (v1p/wp unused;
    GPU with ``bins_rm`` only).  raw (with rec): return the exact int64 fixed-point sums (count, sum * scales[1])
    instead of fp64 moments, so ranks can all-reduce integers (also without rec: (sum w*q0 | count, sum w*q1)).
    CPU: the same fixed-point integers as the HIP kernels (fp32 quantisation, int64 sums), so CPU ranks
    traverse the exact arithmetic of the GPU path."""
    if out is not None:
        assert rec and raw and out.dtype == torch.int64 and out.is_contiguous()
    if rec:
        return _seg_hist_rec(bins, d, B, perm, segs, S, wmax, scales, bins_rm, interleave, raw, out, rm_s10, cls3)
    assert not rm_s10
    return _seg_hist(bins, d, B, perm, v0p, v1p, wp, segs, S, wmax, scales, bins_rm, interleave, raw)


def _seg_flat_index(bins: torch.Tensor, d: int, B: int, rows: torch.Tensor, slot: torch.Tensor) -> torch.Tensor:
    """CPU: flat cell index slot * d * B + f * B + bin(row, f) of every (row, feature) pair, [m, d]."""
    G, n, _ = bins.shape
    flat = bins.permute(1, 0, 2).reshape(n, G * 8)[:, :d].long()
    return slot[:, None] * (d * B) + torch.arange(d)[None, :] * B + flat[rows]


def _int_hist_cpu(bins, d, B, S, rows, slot, *cols) -> torch.Tensor:
    """CPU: exact int64 sums of per-item integers (a0, a1[, a2]) into cells [S, d, B, len(cols)]."""
    k = len(cols)
    out = torch.zeros(S * d * B * k, dtype=torch.int64)
    if rows.numel():
        idx = _seg_flat_index(bins, d, B, rows, slot) * k
        for j, a in enumerate(cols):
            out.index_add_(0, idx.reshape(-1) + j, a[:, None].expand(-1, d).reshape(-1))
    return out.view(S, d, B, k)


def _seg_items(segs: np.ndarray):
    """segs [k, 3] {start, len, slot} -> (item positions, item slots) as int64 tensors."""
    segs = np.asarray(segs, dtype=np.int64).reshape(-1, 3)
    segs = segs[segs[:, 1] > 0]
    if len(segs) == 0:
        return torch.zeros(0, dtype=torch.int64), torch.zeros(0, dtype=torch.int64)
    ln = segs[:, 1]
    pos = np.repeat(segs[:, 0], ln) + (np.arange(int(ln.sum())) - np.repeat(np.cumsum(ln) - ln, ln))
    return torch.from_numpy(pos), torch.from_numpy(np.repeat(segs[:, 2], ln))


def _quant(v: torch.Tensor, scale: float, clamp: bool) -> torch.Tensor:
    """The kernels' fixed-point quantisation: rintf(v * scale) in fp32 (clamped to +-2^23 when packed)."""
    q = torch.round(v.float() * torch.tensor(scale, dtype=torch.float32)).to(torch.int64)
    return q.clamp(-(1 << 23), 1 << 23) if clamp else q


# 3-class packed records (seg.hip kClsSplit): class c's label code is 0 / 1 / CLS3_CODE, so a histogram block's
# sum w * q is W1 + 2^22 W2 (W1 < 2^22 inside a block); the kernels' flush splits it into two int64 columns, so the
# level histograms are [S, d, B, 3] (W, W1, W2) and their global sums have no size bound (round 5 packed
# W1 + 2^32 W2 in one column: n_global * 255 < 2^32 rows at most)
CLS3_CODE = 1 << 22


def hist_cols(cls3: bool) -> int:
    """Int64 columns per cell of a record histogram: (count, sum), or (W, W1, W2) for 3-class records."""
    return 3 if cls3 else 2


def cls3_expand(Hb: torch.Tensor) -> torch.Tensor:
    """3-class record sums [..., 3] (W, W1, W2) -> exact int64 class counts [..., 3] (W0, W1, W2)."""
    W, W1, W2 = Hb[..., 0], Hb[..., 1], Hb[..., 2]
    return torch.stack([W - W1 - W2, W1, W2], -1)


def rec_decode(rec: torch.Tensor):
    """Packed item records -> (row, weight, quantised label) int64 tensors."""
    r = rec.to(torch.int64)
    return r & ((1 << 31) - 1), (r >> 31) & 0xFF, ((r >> 39) & ((1 << 25) - 1)) - (1 << 23)


def rec_encode(rows: torch.Tensor, w: torch.Tensor, q: torch.Tensor) -> torch.Tensor:
    return rows.to(torch.int64) | (w.to(torch.int64) << 31) | ((q.to(torch.int64) + (1 << 23)) << 39)


def _seg_hist_rec(bins, d, B, rec, segs, S, wmax, scales, bins_rm, interleave, raw=False, out=None, rm_s10=False,
                  cls3=False):
    G, n, _ = bins.shape
    segs = np.asarray(segs, dtype=np.int64).reshape(-1, 3)
    kc = hist_cols(cls3)
    if S == 0 or len(segs) == 0:
        if out is not None:
            return out
        return torch.zeros((S, d, B, kc), dtype=torch.int64 if raw else torch.float64, device=bins.device)
    qs1 = float(scales[1])
    if not _native(bins):
        pos, slot = _seg_items(segs)
        rows, w, q = rec_decode(rec[pos])
        if cls3:
            iout = _int_hist_cpu(bins, d, B, S, rows, slot, w, w * (q & (CLS3_CODE - 1)), w * (q >> 22))
        else:
            iout = _int_hist_cpu(bins, d, B, S, rows, slot, w, w * q)
        if out is not None:
            iout = out.copy_(iout)
    else:
        assert bins_rm is not None and rec.dtype == torch.int64
        wm = int(max(1, min(255, wmax)))
        cap = (1 << 20) // (wm + 1)
        if rm_s10 and LANE10_CHUNK3:
            # the six-items-per-wave kernel spreads a block's items over three copies of every cell (item i of the
            # chunk -> copy i % 3): each copy's 20-bit count holds a third of the chunk
            cap = 3 * cap - 1024
        top = SEG_HIST_CHUNK * (3 if rm_s10 and LANE10_CHUNK3 else 1)
        if rm_s10 and int(segs[:, 1].sum()) > 2 * LANE10_CHUNK_MAX * SEG_MIN_BLOCKS:
            # large levels only: the smaller levels of a shard keep _fill_chunk's round fitting (its chunks grow
            # to drop a sliver round; capping them cost +0.25 ms at 1.25e7 rows)
            top = min(top, LANE10_CHUNK_MAX)
        ncu = _num_cus(bins.device) if (SEG_ROUND_FIT and rm_s10 and bins.is_cuda) else 0
        if NATIVE_PLAN:
            chunk, work = _seg_plan(segs, min(top, cap), B, ncu, interleave)
        else:
            chunk = _fill_chunk(segs, min(top, cap), B, ncu)
            work = _seg_work(segs, chunk, interleave)
        if len(work) == 0:
            if out is not None:
                return out
            return torch.zeros((S, d, B, kc), dtype=torch.int64 if raw else torch.float64, device=bins.device)
        wt, = upload(bins.device, work.reshape(-1))
        iout = out if out is not None else torch.zeros((S, d, B, kc), dtype=torch.int64, device=bins.device)
        assert iout.shape == (S, d, B, kc)
        assert bins_rm.shape[0] == n and bins_rm.shape[1] >= G and bins_rm.is_contiguous()
        mode = 1 | 4 | 16 | (128 if (SEG_LANE and B <= SEG_LANE_MAX_B) else 0) | (512 if cls3 else 0)
        if rm_s10:
            assert d <= 100 and B <= 40 and bins_rm.shape[1] == 16
            mode |= 128 | 256
        _lib.check(_lib.lib().cdna_seg_hist(mode, _ptr(bins_rm), n, d, B, _ptr(rec), None, None, None,
                                            _ptr(wt), len(work), 1.0, qs1, _ptr(iout), bins_rm.shape[1],
                                            _stream(bins.device)), "cdna_seg_hist(rec)")
    if raw:
        return iout
    out = iout.double()
    out[..., 1] /= qs1
    return out


CODES_HIST_BLOCKS = 0
CODES_ROUND_FILL = True
_NCU = {}


def _num_cus(dev) -> int:
    if dev.index not in _NCU:
        _NCU[dev.index] = int(torch.cuda.get_device_properties(dev).multi_processor_count)
    return _NCU[dev.index]


def seg_hist_codes(bins_s10: torch.Tensor, d: int, B: int, codes: torch.Tensor, v1: torch.Tensor, qs1: float,
                   wmax: int, slot_tree: np.ndarray, slot_node: np.ndarray, s0: int, s1: int,
                   out: torch.Tensor, draw: Optional[tuple] = None, cls3: bool = False) -> torch.Tensor:
    """Record histograms of slots [s0, s1) straight from the row codes (GPU, seg10 rows), for levels with at most
    one built node per tree: slot s is local node ``slot_node[s]`` of tree ``slot_tree[s]`` (level 0: every root,
    node 0).  Adds the exact int64 sums (count, sum w * q) into ``out`` [s1 - s0, d, B, 2] (zeroed by the caller)
    -- the same integers as ``codes_compact(rec_scale=qs1)`` + ``seg_hist(rec=True, raw=True)``, without
    materialising the level's 8-byte records.

    draw (level 0 of a bootstrapped forest, B <= 40): ``(seed, row offset, rate)`` -- the kernel draws every row's
    Poisson weight itself and WRITES ``codes`` (the lazy :class:`BootstrapCodes`); ``wmax`` must then be the draws'
    static bound (``poisson_max_draw``)."""
    T, n = codes.shape
    wide = 80 < B <= 256
    # B <= 40: seg10 rows, six-items-per-wave kernel; 80 < B <= 256 (boosting): standard row-major rows, lane4
    assert _native(codes) and ((d <= 100 and B <= 40 and bins_s10.shape == (n, 16, 8)) or
                               (wide and bins_s10.shape[0] == n and bins_s10.shape[1] * 8 >= d and
                                bins_s10.is_contiguous()))
    assert out.dtype == torch.int64 and out.is_contiguous() and out.shape == (s1 - s0, d, B, hist_cols(cls3))
    st = np.asarray(slot_tree, dtype=np.int64)
    sn = np.asarray(slot_node, dtype=np.int64)
    assert len(st) == len(sn) and np.all((st >= 0) & (st < T)) and np.all((sn >= 0) & (sn < 0xFF))
    assert len(np.unique(st[s0:s1])) == s1 - s0  # one built node per tree
    if n == 0 or s1 <= s0:
        return out
    wm = int(max(1, min(255, wmax)))
    sinfo = np.stack([st, sn], 1).astype(np.int32).reshape(-1)
    v1c = v1.float().contiguous()
    key = (n, d, B, wm, s0, s1, wide, str(codes.device), CODES_HIST_BLOCKS, CODES_ROUND_FILL)
    work = _ROOT_WORK.get(key)
    if work is None:
        work = _root_work(n, d, wide, wm, s0, s1, codes.device)
        if len(_ROOT_WORK) > 64:
            _ROOT_WORK.clear()
        _ROOT_WORK[key] = work
    if wide:
        wt, si = upload(codes.device, work.reshape(-1), sinfo)
        _lib.check(_lib.lib().cdna_seg_hist_root_wide(_ptr(bins_s10), n, d, B, bins_s10.shape[1] * 8, _ptr(codes),
                                                      _ptr(v1c), float(qs1), _ptr(wt), len(work), _ptr(si), s0,
                                                      _ptr(out), int(cls3), _stream(codes.device)),
                   "cdna_seg_hist_root_wide")
        return out
    wt, si = upload(codes.device, work.reshape(-1), sinfo)
    if draw is not None:
        assert np.array_equal(np.sort(st[s0:s1]), np.arange(T)) and not np.any(sn[s0:s1]), "draws need every root"
    seed, off, rate = draw if draw is not None else (0, 0, 1.0)
    _lib.check(_lib.lib().cdna_seg_hist_root(_ptr(bins_s10), n, d, B, _ptr(codes), _ptr(v1c), float(qs1), _ptr(wt),
                                             len(work), _ptr(si), s0, _ptr(out), int(draw is not None),
                                             int(seed) & 0xFFFFFFFFFFFFFFFF, int(off), float(rate), int(cls3),
                                             _stream(codes.device)),
               "cdna_seg_hist_root")
    return out


# (shape, slot range, device) -> the root / codes histogram work list: the same for every fit of a shard, so its
# host planning (~100 us of numpy per level, on the critical path between a level's decisions and the next level's
# first launch at the per-rank shape) runs once
_ROOT_WORK: Dict[tuple, np.ndarray] = {}


def _root_work(n: int, d: int, wide: bool, wm: int, s0: int, s1: int, device) -> np.ndarray:
    """Work items [m, 3] {row start, rows, slot} of a codes histogram over slots [s0, s1) (see seg_hist_codes)."""
    # each LDS cell copy takes every third item of a wave's stream: rows x wmax / 3 (+ a partial trip per
    # wave) stays below the 20-bit count field (the wide kernel has one copy: rows x wmax)
    rows = max(64, min(n, (1 << 20) // (wm + 1) - 64 if wide else 3 * ((1 << 20) // (wm + 1)) - 16 * 64))
    # CODES_HIST_BLOCKS > 0: shrink the row chunks toward that many blocks (>= 16k rows each).  Off by
    # default: at the per-rank 1.25e7 shape 4096 blocks ran 21.0-21.3 ms per step vs 20.0-20.1 ms with the
    # largest chunks (the per-block LDS clear + flush of 100 KB outweighs the emptier last round)
    S_l = max(1, s1 - s0)
    if CODES_HIST_BLOCKS > 0:
        rows = max(min(rows, 16384), min(rows, -(-(n * S_l) // CODES_HIST_BLOCKS)))
    rows = (rows + 63) // 64 * 64
    C = (n + rows - 1) // rows
    bpc = S_l * (-(-d // 64) if wide else 1)  # blocks per row chunk (the wide kernel: one per 64 features)
    if device.type == "cuda":
        # at least two rounds of blocks (one block per CU) while blocks keep >= 4096 rows: a boosting level of
        # 1.25e7 rows in 524k-row chunks would run 48 blocks on 256 CUs
        C_min = min(-(-2 * _num_cus(device) // bpc), max(1, n // 4096))
        if C < C_min:
            C = C_min
            rows = (-(-n // C) + 63) // 64 * 64
            C = (n + rows - 1) // rows
    if CODES_ROUND_FILL and C * bpc < 64 * _num_cus(device):
        # one block per CU: spread the rows over as many chunks as the rounds of blocks already needed can hold,
        # so the last round is full instead of a fraction of the chip (1.25e7 rows x 20 trees: 640 blocks in 2.5
        # rounds -> 760 in 2.97, 19.2 -> 18.9 ms per step; an exact multiple of the CUs, 1280 blocks in 5
        # rounds, pays each block's 100 KB LDS clear + flush twice as often)
        ncu = _num_cus(device)
        rounds = -(-(C * bpc) // ncu)
        C2 = max(C, (rounds * ncu) // bpc)
        if C2 > C:
            rows = (-(-n // C2) + 63) // 64 * 64
            C = (n + rows - 1) // rows
    # XCD-aware order: block b runs on XCD b % 8; the slots (trees) of row chunk c are consecutive blocks of
    # XCD c % 8, so their row-line gathers and label reads share that XCD's L2
    nq = (C + 7) // 8
    cq, sl, x = np.meshgrid(np.arange(nq), np.arange(s0, s1), np.arange(8), indexing="ij")  # (cq, slot, x) order
    c = (cq * 8 + x).reshape(-1)
    keep = c < C
    c, sl = c[keep], sl.reshape(-1)[keep]
    r0 = c * rows
    work = np.stack([r0, np.minimum(rows, n - r0), sl], 1).astype(np.int32)
    if wide:
        # the kernel pairs the feature blocks of each item on one XCD itself: items in (chunk, slot) order
        work = work[np.lexsort((work[:, 2], work[:, 0]))]
    return work


def seg_hist_root(bins_s10: torch.Tensor, d: int, B: int, codes: torch.Tensor, v1: torch.Tensor, qs1: float,
                  wmax: int, t0: int, t1: int, out: torch.Tensor) -> torch.Tensor:
    """Level 0: :func:`seg_hist_codes` with slot t = the root (local node 0) of tree t, slots [t0, t1)."""
    T = codes.shape[0]
    return seg_hist_codes(bins_s10, d, B, codes, v1, qs1, wmax, np.arange(T), np.zeros(T, np.int64), t0, t1, out)


def _seg_hist(bins: torch.Tensor, d: int, B: int, perm: torch.Tensor, v0p: Optional[torch.Tensor],
              v1p: torch.Tensor, wp: Optional[torch.Tensor], segs: np.ndarray, S: int, wmax: int,
              scales=None, bins_rm: Optional[torch.Tensor] = None, interleave: bool = False,
              raw: bool = False) -> torch.Tensor:
    """Moments [S, d, B, 2] of node segments of ``perm`` (row ids grouped by node).

    segs: [k, 3] {start, len, slot}.  [..., 0] = sum w*v0 (or sum w when v0p is None), [..., 1] = sum w*v1.
    interleave: order the work items by their relative position inside their segment, so that segments
    of different trees (whose rows are all sorted by row id) gather the same region of the bins at the
    same time and share it through L2 / MALL.
    raw: return the int64 fixed-point sums (stat k scaled by ``scales[k]``; stat 0 unscaled when packed).
    """
    G, n, _ = bins.shape
    segs = np.asarray(segs, dtype=np.int64).reshape(-1, 3)
    packed = v0p is None
    wm = int(max(1, min(255, wmax)))
    zero = lambda: torch.zeros((S, d, B, 2), dtype=torch.int64 if raw else torch.float64,  # noqa: E731
                               device=bins.device)
    if S == 0 or len(segs) == 0:
        return zero()
    qs0, qs1 = scales if scales is not None else seg_scales(v0p, v1p, wm, n)
    if not _native(bins):
        pos, slot = _seg_items(segs)
        rows = perm[pos].long()
        w = torch.ones(len(pos), dtype=torch.int64) if wp is None else wp[pos].to(torch.int64)
        if packed:
            a0, a1 = w, w * _quant(v1p[pos], qs1, True)
        else:
            a0, a1 = w * _quant(v0p[pos], qs0, False), w * _quant(v1p[pos], qs1, False)
        iout = _int_hist_cpu(bins, d, B, S, rows, slot, a0, a1)
    else:
        chunk = SEG_HIST_CHUNK if not packed else min(SEG_HIST_CHUNK, (1 << 20) // (wm + 1))
        chunk = _fill_chunk(segs, chunk, B)
        work = _seg_work(segs, chunk, interleave)
        if len(work) == 0:
            return zero()
        wt, = upload(bins.device, work.reshape(-1))
        iout = torch.zeros((S, d, B, 2), dtype=torch.int64, device=bins.device)
        mode =(1 if packed else 0) | (2 if wp is not None else 0) | (4 if bins_rm is not None else 0)
        if bins_rm is not None:
            assert bins_rm.shape[0] == n and bins_rm.shape[1] >= G and bins_rm.is_contiguous()
        src = bins if bins_rm is None else bins_rm
        _lib.check(_lib.lib().cdna_seg_hist(mode, _ptr(src), n, d, B, _ptr(perm), _ptr(v0p), _ptr(v1p), _ptr(wp),
                                            _ptr(wt), len(work), float(qs0), float(qs1), _ptr(iout),
                                            0 if bins_rm is None else bins_rm.shape[1], _stream(bins.device)),
                   "cdna_seg_hist")
    if raw:
        return iout
    out = iout.double()
    if not packed:
        out[..., 0] /= qs0
    out[..., 1] /= qs1
    return out


def seg_partition(bins: torch.Tensor, perm: Optional[torch.Tensor], v0p: Optional[torch.Tensor], v1p: torch.Tensor,
                  wp: Optional[torch.Tensor], segs: np.ndarray, split_feat: np.ndarray, split_bin: np.ndarray,
                  cat_off: np.ndarray, cat_mask: np.ndarray, child: np.ndarray, n_next: int):
    """Stable split of every node segment into its children's segments (rows of leaves dropped).

    segs [A, 2] {start, len} of the active nodes (in active order); child [2A] next-level node index
    or -1; n_next = number of next-level nodes.  Returns (perm, v0p, v1p, wp, segs_next [n_next, 2]).

    ``perm=None`` is the level-0 entry of multi-tree segment mode: active node a is the root of tree
    a over all n rows, ``wp`` is the [T, n] bootstrap weight matrix, ``v0p``/``v1p`` are the unpermuted
    per-row statistics, and rows whose weight in that tree is 0 are dropped.
    """
    G, n, _ = bins.shape
    segs = np.asarray(segs, dtype=np.int64).reshape(-1, 2)
    A = len(segs)
    dev = v1p.device
    sf = np.asarray(split_feat, dtype=np.int32)
    implicit = perm is None
    if implicit:
        assert wp is not None and wp.shape == (A, n) and wp.is_contiguous(), "implicit entry needs [T, n] weights"
        assert np.array_equal(segs[:, 0], np.arange(A) * n) and np.all(segs[:, 1] == n)
        assert A * n < 2 ** 31, "multi-tree segment mode indexes rows with int32"
    if not _native(bins):
        flat = bins.permute(1, 0, 2).reshape(n, G * 8)
        pieces = [[] for _ in range(max(n_next, 0))]
        for a in range(A):
            s, ln = segs[a]
            if ln == 0 or sf[a] < 0:
                continue
            idx = torch.arange(int(s), int(s + ln))
            if implicit:
                rows = idx - a * n
                keep = wp[a].cpu() > 0
                idx, rows = idx[keep], rows[keep]
            else:
                rows = perm[idx].long()
            bv = flat[rows, int(sf[a])].long()
            if cat_off[a] >= 0:
                m = torch.from_numpy(np.asarray(cat_mask, dtype=np.int64).reshape(-1, 8)[cat_off[a]] & 0xFFFFFFFF)
                left = ((m[bv >> 5] >> (bv & 31)) & 1).bool()
            else:
                left = bv <= int(split_bin[a])
            for side, sel in ((0, left), (1, ~left)):
                c = int(child[2 * a + side])
                if c >= 0:
                    pieces[c].append(idx[sel])
        order = [torch.cat(p) if p else torch.zeros(0, dtype=torch.long) for p in pieces]
        lens = np.array([len(o) for o in order], dtype=np.int64)
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]]) if n_next else np.zeros(0, np.int64)
        cat = torch.cat(order) if order else torch.zeros(0, dtype=torch.long)
        if implicit:
            rows = cat % n
            return (rows.to(torch.int32).contiguous(), None if v0p is None else v0p[rows].contiguous(),
                    v1p[rows].contiguous(), wp.reshape(-1)[cat].contiguous(), np.stack([starts, lens], 1))
        return (perm[cat].contiguous(), None if v0p is None else v0p[cat].contiguous(), v1p[cat].contiguous(),
                None if wp is None else wp[cat].contiguous(), np.stack([starts, lens], 1))
    # native: pass 1 counts left/right rows per chunk, host computes output offsets, pass 2 scatters
    tags = np.arange(A, dtype=np.int64)
    work = _seg_work(np.concatenate([segs, tags[:, None]], 1), SEG_PART_CHUNK)
    nw = len(work)
    L = _lib.lib()
    cm = np.asarray(cat_mask, dtype=np.int32).reshape(-1)
    sf_t, sb_t, co_t, cm_t, wt = upload(dev, sf, np.asarray(split_bin, dtype=np.int32),
                                        np.asarray(cat_off, dtype=np.int32), cm if cm.size else np.zeros(8, np.int32),
                                        work.reshape(-1))
    lrc = torch.zeros((2, max(nw, 1)), dtype=torch.int32, device=dev)
    impl_n = n if implicit else 0
    if nw:
        _lib.check(L.cdna_seg_partition(1, _ptr(bins), n, _ptr(perm), None, None, _ptr(wp) if implicit else None,
                                        _ptr(wt), nw, _ptr(sf_t), _ptr(sb_t), _ptr(co_t), _ptr(cm_t), None, None,
                                        _ptr(lrc[0]), None, None, None, None, impl_n, _ptr(lrc[1]), _stream(dev)),
                   "cdna_seg_partition(count)")
    lrc_h = lrc.cpu().numpy()[:, :nw].astype(np.int64)
    lc_h, rc_h = lrc_h[0], lrc_h[1]
    wseg = work[:, 2].astype(np.int64)
    child = np.asarray(child, dtype=np.int64)
    # child sizes
    lens = np.zeros(n_next, dtype=np.int64)
    cl, cr = child[2 * wseg], child[2 * wseg + 1]
    splits = sf[wseg] >= 0
    np.add.at(lens, cl[splits & (cl >= 0)], lc_h[splits & (cl >= 0)])
    np.add.at(lens, cr[splits & (cr >= 0)], rc_h[splits & (cr >= 0)])
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]) if n_next else np.zeros(0, np.int64)
    # per-chunk offsets: child start + rows of the same child in earlier chunks of the segment
    # (work items are in segment order: exclusive scans restart at each segment's first chunk)
    first = np.searchsorted(wseg, wseg, side="left")
    ex_l = np.cumsum(lc_h) - lc_h
    ex_r = np.cumsum(rc_h) - rc_h
    off_l = ex_l - ex_l[first]
    off_r = ex_r - ex_r[first]
    lb = np.where(splits & (cl >= 0), starts[np.maximum(cl, 0)] + off_l, -1) if n_next else np.full(nw, -1)
    rb = np.where(splits & (cr >= 0), starts[np.maximum(cr, 0)] + off_r, -1) if n_next else np.full(nw, -1)
    total = int(lens.sum())
    assert total < 2 ** 31
    perm_o = torch.empty(total, dtype=torch.int32, device=dev)
    v1_o = torch.empty(total, dtype=torch.float32, device=dev)
    v0_o = None if v0p is None else torch.empty(total, dtype=torch.float32, device=dev)
    w_o = None if wp is None else torch.empty(total, dtype=torch.uint8, device=dev)
    if nw and total:
        lb_t, rb_t = upload(dev, lb.astype(np.int32), rb.astype(np.int32))
        _lib.check(L.cdna_seg_partition(2, _ptr(bins), n, _ptr(perm), _ptr(v0p), _ptr(v1p), _ptr(wp), _ptr(wt), nw,
                                        _ptr(sf_t), _ptr(sb_t), _ptr(co_t), _ptr(cm_t), _ptr(lb_t), _ptr(rb_t),
                                        None, _ptr(perm_o), _ptr(v0_o), _ptr(v1_o), _ptr(w_o), impl_n, None,
                                        _stream(dev)), "cdna_seg_partition(scatter)")
    return perm_o, v0_o, v1_o, w_o, np.stack([starts, lens], 1)


def codes_compact(codes: torch.Tensor, tfirst: torch.Tensor, build_slot: np.ndarray, S: int,
                  v0: Optional[torch.Tensor], v1: torch.Tensor, rec_scale: Optional[float] = None):
    """Rows of the nodes a level builds, gathered into one segment per histogram slot.

    codes [T, n] row records (weight << 8 | local node); tfirst [T] first active index per tree;
    build_slot [A] slot of active node a (-1: not built).  Returns (perm int32, v0p, v1p, wp uint8,
    segs [S, 2] {start, len}).  Row order inside a segment is unspecified (the segment histograms
    are exact fixed-point sums, so it does not change any result).

    rec_scale (GPU, no v0, wave-owned path only): return packed int64 item records instead, as
    (rec, None, None, None, segs) with rec = row | w << 31 | (clamp(rint(v1 * rec_scale), +-2^23) + 2^23) << 39.
    """
    T, n = codes.shape
    dev = codes.device
    A = len(build_slot)
    bs = np.asarray(build_slot, dtype=np.int32)
    if not _native(codes):
        c = codes.to(torch.int32) & 0xFFFF
        loc = c & 0xFF
        ids = tfirst.to(torch.int64).to(dev)[:, None] + loc.long()
        slot_t = torch.from_numpy(np.concatenate([bs, [-1]])).to(dev)
        ids = torch.where(loc == CODE_DONE, torch.full_like(ids, A), ids).clamp_max(A)
        slot = slot_t[ids]  # [T, n]
        flat = slot.reshape(-1)
        keep = torch.nonzero(flat >= 0).flatten()
        order = keep[torch.argsort(flat[keep], stable=True)]
        rows = order % n
        lens = np.bincount(flat[keep].numpy(), minlength=S)[:S].astype(np.int64)
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]]) if S else np.zeros(0, np.int64)
        wts = c.reshape(-1)[order] >> 8
        if rec_scale is not None and v0 is None and n < 2 ** 31:
            # the packed item records of the HIP compaction (same fp32 quantisation)
            return rec_encode(rows, wts, _quant(v1[rows], rec_scale, True)), None, None, None, \
                np.stack([starts, lens], 1)
        return (rows.to(torch.int32), None if v0 is None else v0[rows].float(), v1[rows].float(),
                wts.to(torch.uint8), np.stack([starts, lens], 1))
    L = _lib.lib()
    assert tfirst.numel() == T
    # built nodes per tree -> wave-owned kernel when few (stable, no atomics)
    tf_h = tfirst.cpu().numpy().astype(np.int64)
    tree_of = np.searchsorted(tf_h, np.arange(A), side="right") - 1
    built = bs >= 0
    nb_t = np.bincount(tree_of[built], minlength=T) if A else np.zeros(T, np.int64)
    kb_need = int(nb_t.max()) if T else 0
    if 0 < kb_need <= 16 and COMPACT_W:
        return _codes_compact_w(codes, tf_h.astype(np.int32), bs, tree_of, built, nb_t, kb_need, S, v0, v1,
                                rec_scale if (v0 is None and n < 2 ** 31) else None)
    tf, bs_t = upload(dev, tf_h.astype(np.int32), bs)
    v1c = v1.float().contiguous()
    v0c = None if v0 is None else v0.float().contiguous()
    cnt = torch.zeros(max(S, 1), dtype=torch.int32, device=dev)
    _lib.check(L.cdna_codes_compact(1, _ptr(codes), n, T, A, _ptr(tf), _ptr(bs_t), _ptr(v0c), _ptr(v1c), _ptr(cnt),
                                    None, None, None, None, None, 0.0, _stream(dev)), "cdna_codes_compact(count)")
    lens = cnt.cpu().numpy()[:S].astype(np.int64)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]) if S else np.zeros(0, np.int64)
    total = int(lens.sum())
    assert total < 2 ** 31
    rec = rec_scale is not None and v0 is None and n < 2 ** 31
    if rec:
        perm = torch.empty(total + REC_PAD, dtype=torch.int64, device=dev)[:total]  # readable tail
        v1p = v0p = wp = None
    else:
        perm = torch.empty(total, dtype=torch.int32, device=dev)
        v1p = torch.empty(total, dtype=torch.float32, device=dev)
        v0p = None if v0 is None else torch.empty(total, dtype=torch.float32, device=dev)
        wp = torch.empty(total, dtype=torch.uint8, device=dev)
    if total:
        cur, = upload(dev, np.concatenate([starts, [0]]).astype(np.int32))
        _lib.check(L.cdna_codes_compact(2, _ptr(codes), n, T, A, _ptr(tf), _ptr(bs_t), _ptr(v0c), _ptr(v1c),
                                        _ptr(cur), None if rec else _ptr(perm), _ptr(v0p), _ptr(v1p), _ptr(wp),
                                        _ptr(perm) if rec else None, float(rec_scale) if rec else 0.0,
                                        _stream(dev)), "cdna_codes_compact(scatter)")
    return perm, v0p, v1p, wp, np.stack([starts, lens], 1)


def node_compact(node: torch.Tensor, w: torch.Tensor, tfirst: np.ndarray, build_slot: np.ndarray, S: int,
                 v1: torch.Tensor, rec_scale: float):
    """The packed item records of the rows of a level's built nodes from node ids (the levels below the u16
    codes: node [T, n] int32 global active index, -1 = done; w [T, n] uint8), one segment per slot ->
    (rec int64, segs [S, 2] {start, len}) -- codes_compact(rec_scale=...)'s output for these rows (the order
    inside a segment is unspecified; the fixed-point histograms do not depend on it)."""
    T, n = node.shape
    dev = node.device
    A = len(build_slot)
    bs = np.asarray(build_slot, dtype=np.int32)
    tf_h = np.asarray(tfirst, dtype=np.int64)
    if not _native(node):
        slot_t = torch.from_numpy(np.concatenate([bs, [-1]]).astype(np.int64))
        ids = torch.where(node >= 0, node.long(), torch.full_like(node, A, dtype=torch.int64)).clamp_max(A)
        slot = slot_t[ids]
        flat = slot.reshape(-1)
        keep = torch.nonzero(flat >= 0).flatten()
        order = keep[torch.argsort(flat[keep], stable=True)]
        rows = order % n
        lens = np.bincount(flat[keep].numpy(), minlength=S)[:S].astype(np.int64)
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]]) if S else np.zeros(0, np.int64)
        wts = w.reshape(-1)[order].to(torch.int64)
        return rec_encode(rows, wts, _quant(v1[rows], rec_scale, True)), np.stack([starts, lens], 1)
    L = _lib.lib()
    nloc = np.diff(np.concatenate([tf_h, [A]])) if T else np.zeros(0, np.int64)
    max_loc = int(nloc.max()) if T else 0
    tf, bs_t = upload(dev, tf_h.astype(np.int32), bs)
    v1c = v1.float().contiguous()
    cnt = torch.zeros(max(S, 1), dtype=torch.int32, device=dev)
    _lib.check(L.cdna_node_compact(1, _ptr(node), _ptr(w), n, T, A, _ptr(tf), _ptr(bs_t), _ptr(v1c), _ptr(cnt), None,
                                   float(rec_scale), max_loc, _stream(dev)), "cdna_node_compact(count)")
    lens = cnt.cpu().numpy()[:S].astype(np.int64)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]) if S else np.zeros(0, np.int64)
    total = int(lens.sum())
    assert total < 2 ** 31
    rec = torch.empty(total + REC_PAD, dtype=torch.int64, device=dev)[:total]  # readable tail
    if total:
        cur, = upload(dev, np.concatenate([starts, [0]]).astype(np.int32))
        _lib.check(L.cdna_node_compact(2, _ptr(node), _ptr(w), n, T, A, _ptr(tf), _ptr(bs_t), _ptr(v1c), _ptr(cur),
                                       _ptr(rec), float(rec_scale), max_loc, _stream(dev)), "cdna_node_compact(scatter)")
    return rec, np.stack([starts, lens], 1)


NODE_COMPACT_MAX_LOC = 1024  # seg.hip kNodeCompactLoc
COMPACT_W = True
# record compaction without a host round trip before the scatter (device segment starts, totals copied back
# behind the scatter kernel)
COMPACT_DEFER = True


# how codes_scatter_w ranks the lanes of one node (seg.hip codes_scatter_w_kernel): 0 = a ballot per node,
# 1 = one DPP prefix scan per 4 nodes (from SCATTER_SCAN_MIN_KB built nodes per tree; KB = 8: 3.54 vs 3.85 ms)
SCATTER_RANK = 1
SCATTER_SCAN_MIN_KB = 4


# waves per tree of the wave-owned compaction (each owns a contiguous row range: per-wave counts, then offsets).
# A/B (round 5): 512 / 1024 / 2048 -> 17.7 / 17.6 / 17.5-17.6 ms at the per-rank shape, 131.2-131.5 vs 129.7-129.8
# ms at the headline for 512 vs 2048
COMPACT_WAVES = 2048
# rows per wave at least (a multiple of 256): small shards keep fewer, longer waves (the per-block node table and
# the per-wave count flush are fixed costs; the queued scatter carries its queue across the wave's trips)
COMPACT_MIN_PER_WAVE = 256


# queued scatter (seg.hip codes_scatter_q_kernel, rank 2): the built row slots queued per wave in LDS and ranked /
# stored in dense groups of 64 (packed records, per_wave <= 65536); identical records to ranks 0 / 1
SCATTER_QUEUE = True
# the queued scatter with its code / label loads one trip ahead (two register sets; rank 3): 120.9 / 120.9 vs
# 121.6 / 121.6 ms per headline step, scatter 7.7 vs ~8.2 ms (profiles/r6/headline_ab.md)
SCATTER_PREFETCH = True


def _scatter_rank(KB: int, rec: bool = False, per_wave: int = 0) -> int:
    if SCATTER_QUEUE and rec and per_wave <= 65536:
        return 3 if SCATTER_PREFETCH else 2
    return 0 if (SCATTER_RANK == 1 and KB < SCATTER_SCAN_MIN_KB) else SCATTER_RANK


def _codes_compact_w(codes, tf_h, bs, tree_of, built, nb_t, kb_need, S, v0, v1, rec_scale=None):
    T, n = codes.shape
    dev = codes.device
    A = len(bs)
    KB = 1
    while KB < kb_need:
        KB *= 2
    # k of each built node inside its tree (slots are numbered tree-major, so slot = first slot of tree + k)
    kmap = np.full(A, -1, dtype=np.int32)
    first_slot = np.zeros(T, dtype=np.int64)
    first_slot[1:] = np.cumsum(nb_t)[:-1]
    kmap[built] = bs[built] - first_slot[tree_of[built]]
    assert np.all(kmap[built] >= 0) and np.all(kmap[built] < KB)
    per_wave = max(COMPACT_MIN_PER_WAVE, -(-n // (COMPACT_WAVES * 256)) * 256)
    Wv = -(-n // per_wave)
    L = _lib.lib()
    tf, kmap_t = upload(dev, tf_h, kmap)
    v1c = v1.float().contiguous()
    v0c = None if v0 is None else v0.float().contiguous()
    wcnt = torch.empty((T, Wv, KB), dtype=torch.int32, device=dev)
    _lib.check(L.cdna_codes_compact_w(1, KB, _ptr(codes), n, T, A, _ptr(tf), _ptr(kmap_t), _ptr(v0c), _ptr(v1c),
                                      per_wave, Wv, _ptr(wcnt), None, None, None, None, None, None, 0.0, None, 0,
                                      _stream(dev)), "cdna_codes_compact_w(count)")
    # per-(tree, node) exclusive scan over the waves in place + node totals, one launch
    tot = torch.empty((T, KB), dtype=torch.int64, device=dev)
    _lib.check(L.cdna_wave_scan(_ptr(wcnt), T, Wv, KB, _ptr(tot), _stream(dev)), "cdna_wave_scan")
    sl = (first_slot[:, None] + np.arange(KB)[None, :])        # slot of (t, k)
    valid = np.arange(KB)[None, :] < nb_t[:, None]
    rec = rec_scale is not None
    if rec and COMPACT_DEFER and n * T < 2 ** 31:
        # No host round trip before the scatter: slots are numbered tree-major with k inside the tree and
        # (t, k) pairs that are not built count 0, so the segment starts are the exclusive prefix of the
        # [T][KB] totals in place -- computed on the device.  The records buffer is sized by the n * T bound
        # (one item per (row, tree)); the totals come back through pinned memory while the scatter runs, and the
        # host builds the segment table (and the caller its histogram work list) behind it instead of idling
        # the GPU for the D2H copy + host work + H2D copy of every level.
        flat = tot.view(-1)
        kstart_t = torch.cumsum(flat, 0) - flat
        tot_p = torch.empty((T, KB), dtype=torch.int64, pin_memory=True)
        tot_p.copy_(tot, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        perm = torch.empty(n * T + REC_PAD, dtype=torch.int64, device=dev)
        _lib.check(L.cdna_codes_compact_w(2, KB, _ptr(codes), n, T, A, _ptr(tf), _ptr(kmap_t), _ptr(v0c), _ptr(v1c),
                                          per_wave, Wv, None, _ptr(wcnt), None, None, None, None, _ptr(perm),
                                          float(rec_scale), _ptr(kstart_t), _scatter_rank(KB, True, per_wave),
                                          _stream(dev)),
                   "cdna_codes_compact_w(scatter)")
        ev.synchronize()
        tot_h = tot_p.numpy()
        lens = np.zeros(S, dtype=np.int64)
        lens[sl[valid]] = tot_h[valid]
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]]) if S else np.zeros(0, np.int64)
        total = int(lens.sum())
        return perm[:total], None, None, None, np.stack([starts, lens], 1)
    tot_h = tot.cpu().numpy()
    lens = np.zeros(S, dtype=np.int64)
    lens[sl[valid]] = tot_h[valid]
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]) if S else np.zeros(0, np.int64)
    total = int(lens.sum())
    assert total < 2 ** 31
    if rec:
        perm = torch.empty(total + REC_PAD, dtype=torch.int64, device=dev)[:total]  # readable tail
        v1p = v0p = wp = None
    else:
        perm = torch.empty(total, dtype=torch.int32, device=dev)
        v1p = torch.empty(total, dtype=torch.float32, device=dev)
        v0p = None if v0 is None else torch.empty(total, dtype=torch.float32, device=dev)
        wp = torch.empty(total, dtype=torch.uint8, device=dev)
    if total:
        kstart = np.zeros((T, KB), dtype=np.int64)
        kstart[valid] = starts[sl[valid]]
        kstart_t, = upload(dev, kstart)
        # wcnt now holds the per-wave exclusive offsets; the scatter pass adds each node's segment start
        _lib.check(L.cdna_codes_compact_w(2, KB, _ptr(codes), n, T, A, _ptr(tf), _ptr(kmap_t), _ptr(v0c), _ptr(v1c),
                                          per_wave, Wv, None, _ptr(wcnt), None if rec else _ptr(perm), _ptr(v0p),
                                          _ptr(v1p), _ptr(wp), _ptr(perm) if rec else None,
                                          float(rec_scale) if rec else 0.0, _ptr(kstart_t),
                                          _scatter_rank(KB, rec, per_wave),
                                          _stream(dev)),
                   "cdna_codes_compact_w(scatter)")
    return perm, v0p, v1p, wp, np.stack([starts, lens], 1)


BINS_RM_PAD = True


def bins_row_major(bins: torch.Tensor, pad: Optional[bool] = None) -> torch.Tensor:
    """[G, n, 8] feature-group-major bins -> row-major [n, Gs, 8] copy.

    pad (default on the GPU when G <= 16): Gs = 16, zero-filled, so every row is one aligned 128-byte line
    (a gathered 104-byte row at d = 100 touched ~1.8 lines)."""
    G, n, _ = bins.shape
    if not _native(bins):
        return bins.permute(1, 0, 2).contiguous()
    pad = BINS_RM_PAD if pad is None else pad
    Gs = 16 if (pad and G <= 16) else G
    out = torch.empty((n, Gs, 8), dtype=torch.uint8, device=bins.device)
    _lib.check(_lib.lib().cdna_bins_row_major(_ptr(bins), n, G, Gs, _ptr(out), _stream(bins.device)),
               "cdna_bins_row_major")
    return out


# ------------------------------------------------------------ K6 (split.hip)
# K6 over exact histograms (split_scan(exact=True)) in the wave-parallel kernel: a wave per feature instead of a
# thread walking every bin, the same winner bit for bit (split.hip split_scan_wave_kernel)
SPLIT_WAVE = True


def split_scan(H: torch.Tensor, nthr: torch.Tensor, masks: Optional[torch.Tensor], kind: int, min_inst: float,
               reg_lambda: float = 1.0, gamma: float = 0.0, min_child_weight: float = 1.0,
               missing_bin: bool = False, exact: bool = False):
    """Best split per node of level histograms H [A, d, B, 2] (fp64) -> (out [A, 8], tot [A, 2]).

    out = (gain, feature, bin, left0, left1, right0, right1, missing-goes-right); gain -inf when no legal split.
    kind 0: variance gain on (weight, sum); kind 1: XGBoost gain on (hess, grad).
    exact: every prefix sum of H is exact in fp64 (int64 fixed point at power-of-two scales below 2^53), so the
    wave-parallel kernel's summation order gives the serial kernel's bits (``SPLIT_WAVE``)."""
    A, d, B, k = H.shape
    assert k == 2 and H.dtype == torch.float64 and _native(H)
    Hc = H.contiguous()
    out = torch.empty((A, 8), dtype=torch.float64, device=H.device)
    tot = torch.empty((A, 2), dtype=torch.float64, device=H.device)
    nt = nthr.to(device=H.device, dtype=torch.int32).contiguous()
    m = None if masks is None else masks.to(device=H.device, dtype=torch.int32).contiguous()
    mw = 0 if m is None else m.shape[1]
    kw = kind | (0x100 if (exact and SPLIT_WAVE) else 0)
    _lib.check(_lib.lib().cdna_split_scan(_ptr(Hc), _ptr(nt), _ptr(m), mw, A, d, B, kw, int(missing_bin),
                                          float(min_inst),
                                          float(reg_lambda), float(gamma), float(min_child_weight), _ptr(out),
                                          _ptr(tot), _stream(H.device)), "cdna_split_scan")
    return out, tot


def split_decode(so: torch.Tensor, tot: torch.Tensor, a_tree: torch.Tensor, T: int, min_inst: float,
                 min_gain: float, can_level: bool, leaf_children: bool, missing_bin: bool = False,
                 leaf_values: Optional[tuple] = None, catm: Optional[torch.Tensor] = None,
                 nthr: Optional[torch.Tensor] = None):
    """K6 decisions [A, >= 7] + node totals -> partition tables on the device (split.hip split_decode_kernel):
    split_feat / split_bin / cat_off [A], masks [A, 8] (bin sets of missing-right splits, cat_off[a] = a),
    child [2A], tfirst_next [T] (int32), the host decode's exact twin.

    leaf_values ("xgb" | "variance", lambda): also "lv" [3A] fp32, the leaf values of the rows' destinations at
    this level (children that are leaves, active nodes that do not split) for the partition's margin update.
    catm [A, 8] int32 + nthr [d] int32 (split_scan_ex): winners on categorical features (nthr < 0) split by the
    node's category bitmask (cat_off[a] = a)."""
    A = so.shape[0]
    dev = so.device
    out = torch.empty(15 * A + T, dtype=torch.int32, device=dev)
    sf, sb, co = out[:A], out[A:2 * A], out[2 * A:3 * A]
    child, pref, tfn = out[3 * A:5 * A], out[5 * A:7 * A], out[7 * A:7 * A + T]
    masks = out[7 * A + T:15 * A + T]
    sc, tc = so.contiguous(), tot.contiguous()
    lv = torch.empty(3 * A, dtype=torch.float32, device=dev) if leaf_values is not None else None
    vk, lam = (1 if leaf_values[0] == "xgb" else 0, float(leaf_values[1])) if leaf_values is not None else (0, 0.0)
    _lib.check(_lib.lib().cdna_split_decode(_ptr(sc), sc.shape[1], _ptr(tc), tc.shape[1], _ptr(a_tree), A, T,
                                            float(min_inst), float(min_gain), int(bool(can_level)),
                                            int(bool(leaf_children)), int(bool(missing_bin)), _ptr(sf), _ptr(sb),
                                            _ptr(co), _ptr(masks), _ptr(child), _ptr(pref), _ptr(tfn), _ptr(lv), vk,
                                            lam, _ptr(None if catm is None else catm.contiguous()),
                                            _ptr(None if nthr is None else nthr.contiguous()), _stream(dev)),
               "cdna_split_decode")
    return {"split_feat": sf, "split_bin": sb, "cat_off": co, "masks": masks.view(A, 8), "child": child,
            "tfirst_next": tfn, "lv": lv}


def split_scan_ex(H: torch.Tensor, nthr: torch.Tensor, masks: Optional[torch.Tensor], kind: str, min_inst: float):
    """K6 for classification impurities and categorical features (split.hip split_scan_ex_kernel).

    H [A, d, B, K] fp64; nthr [d] (< 0: categorical); kind 'variance' (K = 2) / 'gini' / 'entropy'.
    Returns (out [A, 4 + 2K] = gain, feature, position, 0, left[K], right[K]; tot [A, K]; catmask [A, 8] int32 =
    the left categories of a categorical winner)."""
    A, d, B, Kc = H.shape
    assert H.dtype == torch.float64 and _native(H)
    out = torch.empty((A, 4 + 2 * Kc), dtype=torch.float64, device=H.device)
    tot = torch.empty((A, Kc), dtype=torch.float64, device=H.device)
    cm = torch.empty((A, 8), dtype=torch.int32, device=H.device)
    nt = nthr.to(device=H.device, dtype=torch.int32).contiguous()
    m = None if masks is None else masks.to(device=H.device, dtype=torch.int32).contiguous()
    mw = 0 if m is None else m.shape[1]
    kd = {"variance": 0, "gini": 2, "entropy": 3}[kind]
    _lib.check(_lib.lib().cdna_split_scan_ex(_ptr(H.contiguous()), _ptr(nt), _ptr(m), mw, A, d, B, Kc, kd,
                                             float(min_inst), _ptr(out), _ptr(tot), _ptr(cm), _stream(H.device)),
               "cdna_split_scan_ex")
    return out, tot, cm


from .relops import (  # noqa: E402,F401  (the relational ops, also reachable as K.<name>)
    _merge_moments, col_moments, partition_dest, compact_mask, gather_cols, bucket_compact, _key_bits,
    _bits_values, hash_dense_ids, dense_ids, dict_encode, HP_OPS, _ptr_array, pack_keys, _excl_scan_n, _hp_shape,
    hash_groups, _la_groups, ordered_to_double, JoinTable, join_table, join_probe, _grouped, group_sum,
    group_first)

from . import tune as _tune  # noqa: E402  (CDNAML_TUNE overrides of the constants above)
_tune.apply(__import__(__name__, fromlist=["_"]))
