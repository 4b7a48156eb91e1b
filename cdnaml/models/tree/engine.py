"""Level-wise distributed histogram tree learner (SURVEY §2.5.3 A3–A6, §2.9 P2/P9).

One engine for DecisionTree*, RandomForest*, GBT* and the XGBoost-style
GBDT.  Per tree level, for all trees of a forest at once:

  1. ``hist_moments`` / ``hist_classes`` (HIP, LDS-privatised) build the
     per-(node, feature, bin) statistics of this rank's rows;
  2. ONE fused RCCL all-reduce of the level's histogram over xGMI
     (PLANET's treeAggregate, ML 06 - Decision Trees.py:108-110);
  3. the best split of every active node is found on device (prefix sums
     over bins, impurity gain, categorical centroid ordering);
  4. ``partition`` (HIP) moves every row of every tree to its child.

Because the all-reduced histograms are bit-identical on every rank, every
rank makes identical decisions and ends with the same model; no broadcast is
needed.  Bins come from a global quantile sample (all-gathered), so they do
not depend on the GPU count.  Bootstrap weights are Philox-Poisson keyed by
the GLOBAL row id: a forest trained on 1 or 8 GPUs is the same forest.

Histograms accumulate every feature of the smaller child of each split; its
sibling is parent − child (per-node feature subsets of random forests are
applied at split time).
"""
from __future__ import annotations

import functools
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from ...ops import kernels as K
from ...utils import tracing as _tr
from ..util import IllegalArgumentException
from .binning import (BinnedData, ChunkedRows, _binize_src, _global_sample, _make_binned, _resident,  # noqa: F401
                      _seg10_ok, find_thresholds, find_thresholds_t, make_binned)
from .forest import (Forest, _FrozenList, _NODE_FIELDS, _forest_level_ops, _settled_list, freeze_cut)  # noqa: F401

# compact uint16 row records (hist5.hip) instead of int32 node ids + uint8 weights
USE_CODES = True
# single-tree regression fits (boosting rounds, DecisionTree): rows kept grouped by node (seg.hip)
USE_SEG = True
# multi-tree regression forests: level 0 on row records, then rows grouped by (tree, node) segments
USE_MSEG = True
MSEG_L0 = True  # level 0 through segments too
# single-tree packed fits (boosting rounds with unit hessians, DecisionTree) through row records + compaction
MSEG_T1 = True
# binary and 3-class classification forests on the packed record / segment path (class counts from (W, W1)
# sums; 3 classes: (W, W1, W2) int64 columns, K.cls3_expand)
MSEG_CLS = True
# K6 split search in one HIP kernel (split.hip) where it applies; else the torch formulation
NATIVE_SPLIT = True
# segment-mode forests carry one packed 8-byte record per gathered row (row | weight | quantised label)
MSEG_REC = True
# level 0 on seg10 rows: root records compacted inside the histogram kernel (no codes_compact pass)
ROOT_HIST = True
# regression forests (T > 1) deeper than 8 levels: the packed record levels down to 8, then node ids (as binary
# classification); 0 = the node-id histograms from the root (round 3).  RF 20 trees depth 10 at 1e7 x 100:
# 376 -> 88 ms per fit.  One tree keeps the permutation segment path (seg.hip, any depth): 14 ms at depth 12
# against 38 ms switched (profiles/r4/deep_reg_ab.md)
DEEP_REG = True
# per-node feature subsets drawn on the GPU (misc.hip feature_masks_kernel) on levels whose masks have no host
# consumer; 0 = numpy + upload every level
MASKS_DEV = True
# boosting margins updated by the level partitions (ForestTrainer.train(margin=...)) instead of a tree walk
GBDT_MARGIN = True
# multi-rank record histograms: slot chunks whose all-reduces overlap the next chunk's histogram kernel
HIST_OVERLAP = 2
# ... only for level histograms of at least this many bytes: at the 8-GPU point's per-rank shape (1.25e7 rows)
# building a level in 4 / 2 slot chunks cost 22.2 / 20.6 ms per step vs 19.9 ms in one launch (each chunk's
# launch ends in a partly idle round of blocks), while a <= 10 MB RCCL all-reduce over xGMI takes ~0.1-0.2 ms
HIST_OVERLAP_MIN_BYTES = 64 << 20
# take the slot-chunked (overlapped all-reduce) histogram path on one rank too: measures its launch cost at a
# per-rank shape on a 1-GPU box
HIST_OVERLAP_FORCE = False
# Level histograms of at least this many bytes (int64, distributed, regression / XGBoost statistics, no
# categorical features) are reduce-scattered by feature instead of all-reduced: every rank receives the sums of
# d / W features (1/W of an all-reduce's bytes per GPU), runs K6 on its slice, and the per-node winners are
# all-gathered (a few hundred bytes).  Once a fit switches a tree pass over, its later levels stay
# reduce-scattered (sibling subtraction needs the parent's slice).  GBDT at max_bin=256, d=100: levels >= 5.
RS_MIN_BYTES = 4 << 20
# numeric regression levels on row records: decode the split decisions into partition tables on the device and
# queue the partition before the decisions reach the host (no idle device -> host -> device round trip per level)
DEVICE_DECODE = True
# regression forests with a predict heap: the last split level's decisions go straight into a device copy of the
# heap (K.heap_last_level) and the host's handling of that level (the decisions' device -> host copy, the node
# lists) is left to the forest's pending work, which the predictor runs right after launching -- the transform no
# longer waits for the host between the last split scan and the predict (~0.3-0.4 ms of idle GPU per fit)
HEAP_LAST_DEVICE = True


@dataclass
class TreeParams:
    max_depth: int = 5
    max_bins: int = 32
    min_instances: float = 1.0
    min_info_gain: float = 0.0
    impurity: str = "variance"          # variance | gini | entropy | xgb
    num_classes: int = 0
    feature_subset: Optional[int] = None  # features per node (None = all)
    bootstrap: bool = False
    subsampling_rate: float = 1.0
    seed: int = 0
    reg_lambda: float = 1.0
    gamma: float = 0.0
    min_child_weight: float = 1.0
    min_weight_fraction: float = 0.0
    subset_scope: str = "node"          # "node" (Spark / colsample_bynode) or "tree" (colsample_bytree)
    tree_ids: Optional[np.ndarray] = None  # logical id of each forest tree for feature-subset hashing
                                           # (batched many-model fits: tree t of every group hashes as t)


# ============================================================ trainer
def _impurity_from_counts(c: torch.Tensor, kind: str) -> torch.Tensor:
    # classes are summed left to right with every product rounded first (no FMA), the order K6's impurity_c
    # (split.hip) uses, so tied category centroids order the same way on both paths
    W = c.sum(-1)
    p = c / W.clamp_min(1e-300).unsqueeze(-1)
    q = p if kind == "gini" else torch.where(p > 0, torch.log2(p.clamp_min(1e-300)), torch.zeros_like(p))
    s = p[..., 0] * q[..., 0]
    for i in range(1, c.shape[-1]):
        s = s + p[..., i] * q[..., i]
    return 1.0 - s if kind == "gini" else -s


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _built_nodes(w: np.ndarray, a_sib: np.ndarray, a_parent: np.ndarray) -> np.ndarray:
    """Subtraction levels: the active nodes whose histogram is built -- the smaller of two active siblings (ties:
    the first one), the other derived as parent - sibling; a node without an active sibling is built."""
    build = np.ones(len(w), dtype=bool)
    has = np.nonzero((a_sib >= 0) & (a_parent >= 0))[0]
    wa, ws = w[has], w[a_sib[has]]
    lose = (wa > ws) | ((wa == ws) & (has > a_sib[has]))
    build[has[lose]] = False
    return build


class ForestTrainer:
    """Trains T trees level-synchronously over one BinnedData shard per rank."""

    def __init__(self, session, data: BinnedData, params: TreeParams):
        self.session = session
        self.data = data
        self.p = params
        self.comm = session.comm
        self.device = data.bins.device
        self.classification = params.impurity in ("gini", "entropy")
        self.C = params.num_classes if self.classification else 0
        self.stats_k = self.C if self.classification else 2
        # the largest shard over all ranks: every histogram-path decision below is made from values all ranks
        # agree on, so every rank issues the same collectives (count, dtype) whatever its own row count
        self.n_max = data.n_local if not self.comm.distributed else int(
            self.comm.all_reduce_scalar(float(data.n_local), "max"))

    # ------------------------------------------------------------ helpers
    def _mask_base(self, trees: np.ndarray, node_keys: np.ndarray) -> np.ndarray:
        """Per-node uint64 mix of (seed, tree, heap key) that the feature hashes of _feature_masks start from."""
        keys = np.ones(len(trees), dtype=np.uint64) if self.p.subset_scope == "tree" else node_keys.astype(np.uint64)
        with np.errstate(over="ignore"):
            return (np.uint64(self.p.seed & 0xFFFFFFFFFFFF) * np.uint64(0x9E3779B97F4A7C15)
                    + trees.astype(np.uint64) * np.uint64(0xBF58476D1CE4E5B9)
                    + keys * np.uint64(0x94D049BB133111EB))

    def _feature_masks(self, trees: np.ndarray, node_keys: np.ndarray) -> np.ndarray:
        """Feature-subset bit words [A, ceil(d/32)] for a level's nodes (featureSubsetStrategy).

        Node (tree t, heap key) keeps the k features with the smallest splitmix64 hash of
        (seed, t, key, feature): a uniform k-subset per node, drawn for the whole level in a few
        vectorised numpy ops (the per-node Generator took ~40 us per node: 6 ms of host time at
        160 nodes, idling the GPU between levels).  Identical on every rank.
        """
        k = self.p.feature_subset
        d = self.data.d
        A = len(trees)
        words = np.zeros((A, (d + 31) // 32), dtype=np.uint32)
        if k is None or k >= d or A == 0:
            return words
        base = self._mask_base(trees, node_keys)
        with np.errstate(over="ignore"):
            h = _splitmix64(base[:, None] + np.arange(d, dtype=np.uint64)[None, :] * np.uint64(0xD6E8FEB86659FD93))
        feats = np.argpartition(h, k - 1, axis=1)[:, :k]
        rows = np.repeat(np.arange(A), k)
        f = feats.reshape(-1)
        np.bitwise_or.at(words, (rows, f >> 5), (np.uint32(1) << (f & 31).astype(np.uint32)))
        return words

    def _node_stats(self, H: torch.Tensor, fmask_any: torch.Tensor) -> torch.Tensor:
        """Node totals [A, k] from per-feature bin sums (masked features are zero)."""
        per_f = H.sum(2)  # [A, d, k]
        w = per_f[..., 0] if not self.classification else per_f.sum(-1)
        best_f = torch.argmax(w, dim=1)
        return per_f[torch.arange(H.shape[0], device=H.device), best_f]

    def _leaf_value(self, st: np.ndarray) -> np.ndarray:
        if self.classification:
            W = st.sum()
            return st / W if W > 0 else np.full(self.C, 1.0 / max(self.C, 1))
        if self.p.impurity == "xgb":
            H, G = st[0], st[1]
            return np.array([-G / (H + self.p.reg_lambda)])
        W, S = st[0], st[1]
        return np.array([S / W if W > 0 else 0.0])

    def _weights_v(self, st: np.ndarray) -> np.ndarray:
        """Node weights of stats rows [N, k]."""
        if st.shape[0] == 0:
            return np.zeros(0)
        return st.sum(1) if self.classification else st[:, 0].astype(np.float64)

    def _leaf_values_v(self, st: np.ndarray) -> np.ndarray:
        """``_leaf_value`` of stats rows [N, k] -> [N, k_out]."""
        N = st.shape[0]
        if self.classification:
            W = st.sum(1, keepdims=True)
            with np.errstate(invalid="ignore", divide="ignore"):
                return np.where(W > 0, st / np.where(W > 0, W, 1.0), 1.0 / max(self.C, 1))
        if N == 0:
            return np.zeros((0, 1))
        if self.p.impurity == "xgb":
            return (-st[:, 1] / (st[:, 0] + self.p.reg_lambda))[:, None]
        W, S = st[:, 0], st[:, 1]
        return np.where(W > 0, S / np.where(W > 0, W, 1.0), 0.0)[:, None]

    def _impurities_v(self, st: np.ndarray) -> np.ndarray:
        if self.classification and st.shape[0]:
            return _impurity_from_counts(torch.from_numpy(np.ascontiguousarray(st)), self.p.impurity).double().numpy()
        return np.full(st.shape[0], np.nan)

    def _weight(self, st: np.ndarray) -> float:
        return float(st.sum()) if self.classification else float(st[0])

    def _impurity(self, st: np.ndarray) -> float:
        if self.classification:
            t = torch.from_numpy(st)[None]
            return float(_impurity_from_counts(t, self.p.impurity)[0])
        return float("nan")

    # ------------------------------------------------------------ split scan
    def _native_split(self, dev) -> bool:
        """K6 kernel for regression variance / XGBoost gains (incl. missing-value bins), no categoricals."""
        return (NATIVE_SPLIT and dev.type == "cuda" and not self.classification and not self.data.categorical and
                self.stats_k == 2)

    def _native_split_ex(self, dev) -> bool:
        """K6 kernel for classification impurities (<= 32 classes) and categorical features (split_scan_ex)."""
        if not (NATIVE_SPLIT and dev.type == "cuda" and self.data.B <= 256):
            return False
        if self.classification:
            return self.p.impurity in ("gini", "entropy") and 1 <= self.C <= 32
        return self.p.impurity == "variance" and self.stats_k == 2

    def _nthr_dev(self, dev):
        t = getattr(self, "_nthr_t", None)
        if t is None:
            t, = K.upload(dev, np.asarray(self.data.nthr, dtype=np.int32))  # async (a pageable copy drains the queue)
            self._nthr_t = t
        return t

    def _best_splits(self, H: torch.Tensor, tot: torch.Tensor, masks: torch.Tensor, nthr_np=None):
        """H [A, d, B, k] (f64) -> per node (gain, feat, bin, left stats, right stats, cat order)."""
        A, d, B, k = H.shape
        p = self.p
        nthr = torch.from_numpy(self.data.nthr if nthr_np is None else nthr_np).to(H.device)
        cat_feats = sorted(self.data.categorical)
        Hs = H
        order = None
        if cat_feats:
            cf = torch.tensor(cat_feats, device=H.device)
            Hc = H[:, cf]  # [A, nc, B, k]
            if self.classification:
                W = Hc.sum(-1)
                if self.C == 2:
                    cent = Hc[..., 1] / W.clamp_min(1e-300)
                else:
                    cent = _impurity_from_counts(Hc, p.impurity)
            elif p.impurity == "xgb":
                W = Hc[..., 0]
                cent = Hc[..., 1] / (W + p.reg_lambda)
            else:
                W = Hc[..., 0]
                cent = Hc[..., 1] / W.clamp_min(1e-300)
            cent = torch.where(W > 0, cent, torch.full_like(cent, float("inf")))
            order = torch.argsort(cent, dim=-1, stable=True)  # [A, nc, B]
            Hs = H.clone()
            Hs[:, cf] = torch.gather(Hc, 2, order.unsqueeze(-1).expand(-1, -1, -1, k))
        cum = Hs.cumsum(2)
        left = cum
        right = tot[:, None, None, :] - cum
        if self.classification:
            WL, WR = left.sum(-1), right.sum(-1)
            Wt = tot.sum(-1)[:, None, None]
            imp_p = _impurity_from_counts(tot, p.impurity)[:, None, None]
            gain = imp_p - WL / Wt * _impurity_from_counts(left, p.impurity) - \
                WR / Wt * _impurity_from_counts(right, p.impurity)
            valid = (WL >= max(p.min_instances, 1e-12)) & (WR >= max(p.min_instances, 1e-12))
        elif p.impurity == "xgb":
            HL, GL = left[..., 0], left[..., 1]
            HR, GR = right[..., 0], right[..., 1]
            Ht, Gt = tot[:, 0][:, None, None], tot[:, 1][:, None, None]
            lam = p.reg_lambda
            gain = 0.5 * (GL * GL / (HL + lam) + GR * GR / (HR + lam) - Gt * Gt / (Ht + lam)) - p.gamma
            valid = (HL >= p.min_child_weight) & (HR >= p.min_child_weight) & (HL > 0) & (HR > 0)
        else:
            WL, SL = left[..., 0], left[..., 1]
            WR, SR = right[..., 0], right[..., 1]
            Wt, St = tot[:, 0][:, None, None], tot[:, 1][:, None, None]
            gain = (SL * SL / WL.clamp_min(1e-300) + SR * SR / WR.clamp_min(1e-300) - St * St /
                    Wt.clamp_min(1e-300)) / Wt.clamp_min(1e-300)
            valid = (WL >= max(p.min_instances, 1e-12)) & (WR >= max(p.min_instances, 1e-12))
        miss2 = None
        if p.impurity == "xgb" and self.data.missing_bin:
            # option 2: missing rows (bin 0) go RIGHT: left = bins 1..b
            left2 = cum - Hs[:, :, 0:1, :]
            right2 = tot[:, None, None, :] - left2
            HL2, GL2 = left2[..., 0], left2[..., 1]
            HR2, GR2 = right2[..., 0], right2[..., 1]
            gain2 = 0.5 * (GL2 * GL2 / (HL2 + lam) + GR2 * GR2 / (HR2 + lam) - Gt * Gt / (Ht + lam)) - p.gamma
            valid2 = (HL2 >= p.min_child_weight) & (HR2 >= p.min_child_weight) & (HL2 > 0) & (HR2 > 0)
            miss2 = (gain2, valid2, left2, right2)
        # legal split positions per feature
        bpos = torch.arange(B, device=H.device)[None, :]
        limit = torch.where(nthr >= 0, nthr, torch.full_like(nthr, 0))[:, None]  # continuous: b < nthr
        legal = bpos < limit  # [d, B]
        if cat_feats:
            nonempty = (Hc.sum(-1) if self.classification else Hc[..., 0]) > 0  # [A, nc, B]
            ncnt = nonempty.sum(-1)  # [A, nc]
            legal_c = bpos[None, None, :] < (ncnt - 1).unsqueeze(-1)  # [A, nc, B]
            legal_full = legal[None].expand(A, -1, -1).clone()
            legal_full[:, cf] = legal_c
            legal = legal_full
        else:
            legal = legal[None].expand(A, -1, -1)
        valid = valid & legal
        if masks is not None:
            fm = ((masks[:, (torch.arange(d, device=H.device) >> 5)] >>
                   (torch.arange(d, device=H.device) & 31).to(masks.dtype)) & 1).bool()  # [A, d]
            valid = valid & fm[:, :, None]
        gain = torch.where(valid & torch.isfinite(gain), gain, torch.full_like(gain, float("-inf")))
        ar = torch.arange(A, device=H.device)
        if miss2 is not None:
            gain2, valid2, left2, right2 = miss2
            valid2 = valid2 & legal & (bpos >= 1)
            if masks is not None:
                valid2 = valid2 & fm[:, :, None]
            gain2 = torch.where(valid2 & torch.isfinite(gain2), gain2, torch.full_like(gain2, float("-inf")))
            both = torch.cat([gain.reshape(A, -1), gain2.reshape(A, -1)], 1)
            best = torch.argmax(both, dim=1)
            bgain = both[ar, best]
            mr = best >= d * B
            best = best % (d * B)
            bf, bb = best // B, best % B
            lstats = torch.where(mr[:, None], left2[ar, bf, bb], left[ar, bf, bb])
            rstats = torch.where(mr[:, None], right2[ar, bf, bb], right[ar, bf, bb])
            return bgain, bf, bb, lstats, rstats, order, cat_feats, mr
        flat = gain.reshape(A, -1)
        best = torch.argmax(flat, dim=1)
        bgain = flat[ar, best]
        bf = best // B
        bb = best % B
        lstats = left[ar, bf, bb]
        rstats = right[ar, bf, bb]
        return bgain, bf, bb, lstats, rstats, order, cat_feats, None

    # ------------------------------------------------------------ device-side split decode
    def _device_decode_ok(self, dev, use_codes: bool, missing_right: bool) -> bool:
        return (DEVICE_DECODE and dev.type == "cuda" and use_codes and not self.data.categorical and
                not self.classification and self.stats_k == 2)

    @staticmethod
    def _check_decode(dec, split_feat, split_bin, cat_off, cat_masks, child, n_tree, T):
        """Checked build: the device decode equals the host decode the forest was built from (bin sets compared
        by content: the host numbers them densely, the device by node)."""
        tfn = np.searchsorted(n_tree, np.arange(T), side="left").astype(np.int32)
        got = {k: v.cpu().numpy() for k, v in dec.items() if v is not None}
        sp = split_feat >= 0
        ok = (np.array_equal(got["split_feat"], split_feat) and np.array_equal(got["split_bin"][sp], split_bin[sp])
              and np.array_equal(got["child"], child) and np.array_equal(got["tfirst_next"], tfn)
              and np.array_equal(got["cat_off"] >= 0, cat_off >= 0))
        for a in np.nonzero(cat_off >= 0)[0]:
            ok = ok and np.array_equal(got["masks"][a].view(np.uint32), np.asarray(cat_masks[cat_off[a]], np.uint32))
        if not ok:
            raise RuntimeError("device split decode differs from the host decode")

    # ------------------------------------------------------------ device-queued partition
    def _device_partition(self, so, tot, a_tree, tfirst, T, depth, mb, codes, margin=None, catm=None, node=None,
                          pre=None):
        """Partition tables decoded on the device from the level's K6 decisions and the row partition queued right
        behind them (the GPU partitions while the decisions travel to the host; the host repeats the decode to
        build the forest and the next level, checked against the device's in the checked build).  -> the decode
        tables."""
        p, data, dev = self.p, self.data, self.device
        # (``pre``: the two tables uploaded at the level start with the level's other small tables)
        a_tree_d, tf_d = pre if pre is not None else \
            K.upload(dev, a_tree.astype(np.int32), tfirst.numpy().astype(np.int32))
        dec = K.split_decode(so, tot, a_tree_d, T, p.min_instances, p.min_info_gain,
                             depth < p.max_depth, depth + 1 >= p.max_depth, missing_bin=mb,
                             leaf_values=(p.impurity, p.reg_lambda) if margin is not None else None,
                             catm=catm, nthr=self._nthr_dev(dev) if catm is not None else None)
        with _tr.span("tree.partition", depth=depth):
            if node is not None:
                # levels below the u16 codes: the node-id partition from the same device tables (child = the
                # next level's global active index, as the host decode's)
                K.partition(data.bins, node, dec["split_feat"], dec["split_bin"], dec["cat_off"],
                            dec["masks"].reshape(-1), dec["child"])
                return dec
            fm = data.feature_major_bins() if (margin is not None and K.PART_FEATURE_MAJOR) else None
            K.partition_codes(data.bins, codes, tf_d, dec["tfirst_next"], dec["split_feat"],
                              dec["split_bin"], dec["cat_off"], dec["masks"].reshape(-1), dec["child"],
                              margin=(margin[0], dec["lv"], margin[1]) if margin is not None else None,
                              bins_fm=fm)
        return dec

    # ------------------------------------------------------------ reduce-scatter by feature
    def _rs_want(self, Hb: torch.Tensor, rs_on: bool) -> bool:
        if Hb.dtype != torch.int64:
            return False
        return self._rs_level(Hb.numel() * 8, rs_on)

    def _rs_level(self, nbytes: int, rs_on: bool) -> bool:
        """An int64 level histogram of ``nbytes`` is reduce-scattered by feature (not all-reduced)."""
        if not self.comm.distributed or self.data.categorical or self.classification or self.stats_k != 2:
            return False
        return rs_on or nbytes >= RS_MIN_BYTES

    def _reduce_scatter_features(self, Hb: torch.Tensor, d: int):
        """Exact int64 level histograms [S, d, B, k] summed over ranks, this rank keeping features [f0, f1)
        (d / W of them; RCCL reduce_scatter of the feature-major copy)."""
        W, r = self.comm.world_size, self.comm.rank
        dc = -(-d // W)
        S, _, B, k = Hb.shape
        Hp = torch.zeros((W * dc, S, B, k), dtype=Hb.dtype, device=Hb.device)
        Hp[:d] = Hb.permute(1, 0, 2, 3)
        with _tr.span("tree.reduce_scatter", cat="comm", bytes=Hp.numel() * 8 // W):
            mine = self.comm.reduce_scatter(Hp.view(W, -1)).view(dc, S, B, k)
        f0 = min(d, r * dc)
        f1 = min(d, f0 + dc)
        return (f0, f1), mine[: f1 - f0].permute(1, 0, 2, 3).contiguous()

    def _rs_enter(self, st: "_FitState", rs_slice) -> None:
        """A level was reduce-scattered by feature: the pass stays on this rank's feature slice, and the parents'
        histograms (parent - sibling derivation) are cut to it."""
        st.rs_on = True
        if st.prev_hist is not None and st.prev_hist.shape[1] == self.data.d:
            st.prev_hist = st.prev_hist[:, rs_slice[0]:rs_slice[1]].contiguous()

    def _k6_exact(self, st: "_FitState", lv: "_Level") -> bool:
        """The level histograms are exact in fp64: packed int64 sums (|q| <= 2^23 at a power-of-two scale, unit
        count scale) whose totals stay below 2^53 ulps (total weight < 2^30), assembled by exact differences."""
        sc = lv.hist_raw_scale
        return sc is not None and not isinstance(sc, tuple) and self.data.n_global * max(1, st.wmax) < 2 ** 30

    def _rs_split(self, H: torch.Tensor, rs, masks_np, d: int, dev, exact: bool = False):
        """K6 over this rank's feature slice, then the per-node winners of all ranks all-gathered and merged:
        the largest gain, ties to the lowest global candidate key (missing-right * d * B + f * B + b), the
        order one K6 over all features uses -- so the forest is the all-reduce forest bit for bit."""
        p = self.p
        f0, f1 = rs
        A, dl, B = H.shape[0], f1 - f0, H.shape[2]
        if dl > 0:
            mk = None
            if masks_np is not None:
                f = np.arange(f0, f1)
                bits = ((masks_np[:, f >> 5] >> (f & 31).astype(np.uint32)) & 1).astype(np.uint32)
                words = np.zeros((A, -(-dl // 32)), dtype=np.uint32)
                for j in range(dl):
                    words[:, j >> 5] |= bits[:, j] << np.uint32(j & 31)
                mk, = K.upload(dev, words.view(np.int32))
            if self._native_split(dev):
                so, tot = K.split_scan(H, self._nthr_dev(dev)[f0:f1].contiguous(), mk,
                                       1 if p.impurity == "xgb" else 0, p.min_instances, p.reg_lambda, p.gamma,
                                       p.min_child_weight, missing_bin=p.impurity == "xgb" and self.data.missing_bin,
                                       exact=exact)
            else:
                tot = self._node_stats(H, None)
                gain, bf, bb, lst, rst, _, _, mr = self._best_splits(H, tot, mk, self.data.nthr[f0:f1])
                mr = torch.zeros_like(gain) if mr is None else mr.double()
                so = torch.cat([gain[:, None], bf[:, None].double(), bb[:, None].double(), lst, rst, mr[:, None]], 1)
            so = so.clone()
            found = torch.isfinite(so[:, 0])
            so[:, 1] += f0
            key = torch.where(found, so[:, 7] * (d * B) + so[:, 1] * B + so[:, 2],
                              torch.full_like(so[:, 0], float("inf")))
        else:
            so = torch.zeros((A, 8), dtype=torch.float64, device=H.device)
            so[:, 0] = float("-inf")
            tot = torch.zeros((A, 2), dtype=torch.float64, device=H.device)
            key = torch.full((A,), float("inf"), dtype=torch.float64, device=H.device)
        allp = self.comm.all_gather_tensor(torch.cat([so, key[:, None], tot], 1))  # [W, A, 11]
        g, kk = allp[:, :, 0], allp[:, :, 8]
        kk = torch.where(g == g.max(0).values[None], kk, torch.full_like(kk, float("inf")))
        sel = allp[kk.argmin(0), torch.arange(A, device=allp.device)]
        return sel[:, :8].contiguous(), sel[:, 9:11].contiguous()

    # ------------------------------------------------------------ training
    def _hist_overlapped(self, data, d, B, rec, sb, S, wmax, scales, dev, cls3=False, rs=False):
        """Record histograms of a level's S slots in HIST_OVERLAP slot chunks; chunk c's collective runs on the
        collective stream while chunk c + 1 is built (one per-level RCCL collective of 1-50 MB otherwise
        serialises with the compute stream).  The sums are exact integers, so the result is identical to one
        fused collective.

        rs (reduce-scatter by feature, RS_MIN_BYTES levels): each chunk's feature-major copy is reduce-scattered
        asynchronously instead of all-reduced, and the result is this rank's feature slice of all S slots --
        ``(H [S, f1 - f0, B, k], (f0, f1))``, what ``_reduce_scatter_features`` returns for the whole level."""
        kc = K.hist_cols(cls3)
        Hb = torch.zeros((S, d, B, kc), dtype=torch.int64, device=dev)
        k = min(HIST_OVERLAP, S)
        bounds = np.linspace(0, S, k + 1).round().astype(np.int64)
        rm, s10 = data.record_rows() if dev.type == "cuda" else (None, False)
        W, r = self.comm.world_size, self.comm.rank
        dc = -(-d // W)
        pend = []
        for c in range(k):
            s0, s1 = int(bounds[c]), int(bounds[c + 1])
            if s1 <= s0:
                continue
            with _tr.span("tree.hist_chunk", slots=s1 - s0):
                sel = (sb[:, 2] >= s0) & (sb[:, 2] < s1)
                sbc = sb[sel].copy()
                sbc[:, 2] -= s0
                K.seg_hist(data.bins, d, B, rec, None, None, None, sbc, s1 - s0, wmax, scales, bins_rm=rm,
                           interleave=True, rec=True, raw=True, out=Hb[s0:s1], rm_s10=s10, cls3=cls3)
            nbytes = (s1 - s0) * d * B * kc * 8
            if rs:
                Hp = torch.zeros((W * dc, s1 - s0, B, kc), dtype=torch.int64, device=dev)
                Hp[:d] = Hb[s0:s1].permute(1, 0, 2, 3)
                sp = _tr.begin("tree.reduce_scatter", cat="comm", bytes=nbytes // W, slots=s1 - s0)
                pend.append((s0, s1, self.comm.reduce_scatter_async(Hp.view(W, -1)), sp))
            else:
                sp = _tr.begin("tree.allreduce_async", cat="comm", bytes=nbytes, slots=s1 - s0)
                pend.append((s0, s1, self.comm.all_reduce_async(Hb[s0:s1]), sp))
        if not rs:
            with _tr.span("tree.allreduce_wait", cat="comm"):
                for _, _, h, sp in pend:
                    h.wait()
                    _tr.end(sp)
            return Hb
        f0 = min(d, r * dc)
        f1 = min(d, f0 + dc)
        out = torch.empty((S, f1 - f0, B, kc), dtype=torch.int64, device=dev)
        with _tr.span("tree.reduce_scatter_wait", cat="comm"):
            for s0, s1, h, sp in pend:
                mine = h.wait().view(dc, s1 - s0, B, kc)
                _tr.end(sp)
                out[s0:s1] = mine[: f1 - f0].permute(1, 0, 2, 3)
        return out, (f0, f1)

    def train(self, num_trees: int, stats_rows: Dict[str, torch.Tensor], weights: Optional[torch.Tensor],
              forest: Optional[Forest] = None, codes_pre=None, margin=None) -> Forest:
        """Grow ``num_trees`` trees. stats_rows: {'v0','v1'} (moments) or {'label'} (classes).

        codes_pre: a K.BootstrapCodes (the bootstrap draws already written as the row codes) instead of
        ``weights``.
        margin: ``(F [n] fp32, eta)`` (boosting, one tree): when the level loop can, each level's row partition
        also adds ``eta * leaf value`` to F for the rows that finish there (a last partition at the deepest
        level), so the caller needs no tree walk; ``self.margin_applied`` says whether it did.

        Per level (every tree of the forest at once): ``_level_tables`` (which nodes build a histogram, feature
        masks, the level's small device tables), ``_level_histogram`` (HIP record / code / node-id histograms),
        ``_level_reduce`` (one RCCL all-reduce or a reduce-scatter by feature), ``_level_decide`` (histogram
        assembly + K6 split search; the device decode + partition queued behind it where it applies) and
        ``_level_advance`` (the children, the host-side partition paths, the forest bookkeeping)."""
        st = self._fit_paths(num_trees, stats_rows, weights, forest, codes_pre, margin)
        self._fit_rows(st, codes_pre)
        for depth in range(self.p.max_depth + 1):
            if len(st.a_tree) == 0:
                break
            lv = self._level_tables(st, depth)
            with _tr.span("tree.hist", depth=depth, slots=len(lv.build_ids)):
                self._level_histogram(st, lv, depth)
            self._level_reduce(st, lv)
            with _tr.span("tree.split", depth=depth):
                self._level_decide(st, lv, depth)
            if lv.deferred is not None:
                # the last level, decided on the device: its host side runs as the forest's pending work
                st.pending.append(functools.partial(self._level_deferred, st, lv, depth))
                break
            self._level_advance(st, lv, depth)
        return self._fit_finish(st)

    # ------------------------------------------------------------ fit: paths and row state
    def _fit_paths(self, T: int, stats_rows, weights, forest, codes_pre, margin) -> "_FitState":
        """Choose the fit's histogram / partition paths once (they hold for every level but a deep forest's switch
        to node ids) and set up the per-fit state."""
        p, data, dev = self.p, self.data, self.device
        st = _FitState()
        st.T = T
        st.fresh = forest is None
        st.forest = forest or Forest(self.C if self.classification else 1)
        st.forest._heap_np = None
        # single-output forests of depth <= 8 with numeric splits: the predict heap table (Forest.heap_arrays) is
        # filled level by level here, from the keys and values the levels already hold, instead of re-walking the
        # finished forest in Python between the last split and the transform (the GPU idles through that)
        st.heap = st.heap_v = None
        if st.fresh and not self.classification and p.max_depth <= 8 and not data.categorical and \
                not data.missing_bin:
            st.heap = np.zeros((T, 2 ** (p.max_depth + 1) - 1, 2), dtype=np.int32)
            st.heap[:, :, 0] = -1
            st.heap_v = np.zeros((T, 2 ** (p.max_depth + 1) - 1), dtype=np.float64)  # leaf values per slot (fp64)
        st.heap_depth = 0
        st.heap_dev = None  # (device heap, depth, masks) of a deferred last level (_defer_decisions)
        st.need_masks = p.feature_subset is not None and p.feature_subset < data.d
        # several regression trees: row records for every level (one dense pass partitions all trees); before
        # each level's histogram the rows of the nodes it builds are gathered into slot segments, so the
        # histogram touches only those rows
        # binary classification rides the packed regression path: with label y in {0, 1} and scale 1 the packed
        # sums (count, sum w * y) are (W, W1), turned into the class counts (W - W1, W1) in int64 before K6 --
        # exactly the class histograms of the node-id / codes kernels, so the forest does not change.  Forests
        # deeper than 8 levels (u16 codes hold <= 255 nodes per tree) switch to node ids at level 8
        st.cls2 = self.classification and self.C == 2 and MSEG_CLS
        # three classes: label codes 0 / 1 / 2^22 in the records' one quantised value; the histogram kernels split
        # each block's sum W1 + 2^22 W2 into two int64 columns (no bound on the row count), and the codes hold <= 255
        # nodes per tree (no node-id switch below level 8)
        st.cls3 = (self.classification and self.C == 3 and MSEG_CLS and p.max_depth <= 8 and
                   MSEG_REC and stats_rows.get("v0") is None and 8 * data.B * 8 <= 128 * 1024)
        st.deep_switch = (st.cls2 or (not self.classification and DEEP_REG and T > 1)) and p.max_depth > 8
        if st.cls2:
            stats_rows = dict(stats_rows, v1=stats_rows["label"].float())
        elif st.cls3:
            lab = stats_rows["label"]
            stats_rows = dict(stats_rows, v1=torch.where(lab == 2, torch.full_like(lab, K.CLS3_CODE), lab).float())
        st.stats_rows = stats_rows
        # every level builds all features of the smaller child of each split; its sibling is parent - child
        # (feature subsets are applied at split time: the measured alternatives that accumulate only each node's
        # sampled features lost 2-8x, profiles/r3/subhist_ab.md, profiles/pmc_seg_hist_subset.txt)
        st.use_mseg = (USE_MSEG and USE_CODES and (T > 1 or (MSEG_T1 and stats_rows.get("v0") is None)) and
                       (not self.classification or st.cls2 or st.cls3) and (p.max_depth <= 8 or st.deep_switch) and
                       T * self.n_max < 2 ** 31 and data.n_global > 0)
        # one regression tree: rows grouped by node in a permutation (segment mode)
        st.use_seg = USE_SEG and T == 1 and not self.classification and not st.use_mseg
        # row records (uint16 weight<<8 | local node) when every level fits 255 nodes per tree
        st.use_codes = USE_CODES and (p.max_depth <= 8 or (st.deep_switch and st.use_mseg)) and not st.use_seg
        if codes_pre is not None and not st.use_codes:
            weights = codes_pre.weights()  # a path that reads the multiplicities themselves
        st.weights = weights
        # margin updates by the partition need every level on the device decode + partition5 path, every row in
        # the tree (no zero weights) and leaf values the device can form (no categorical / classification)
        st.margin = margin
        st.margin_ok = (margin is not None and GBDT_MARGIN and st.use_codes and not st.deep_switch and T == 1 and
                        weights is None and codes_pre is None and dev.type == "cuda" and p.impurity == "xgb" and
                        self._device_decode_ok(dev, True, False) and self._native_split(dev) and
                        not data.categorical and p.max_depth <= 8)
        self.margin_applied = st.margin_ok
        # packed 8-byte item records (row | weight | quantised label) for the segment histograms
        st.rec_ok = MSEG_REC and stats_rows.get("v0") is None and 8 * data.B * 8 <= 128 * 1024
        # the level's active nodes as a struct of arrays (host): tree, forest id, heap key, stats [A, k],
        # sibling / parent positions (-1 = none).  The per-level host work between the split decisions'
        # device->host copy and the next level's launches is a few vectorised numpy ops, not a per-node
        # Python loop (that loop idled the GPU for 0.2-2.5 ms per level at 20 trees x 2^L nodes)
        st.a_tree = np.arange(T, dtype=np.int32)
        st.a_fid = np.full(T, -1, dtype=np.int64)
        st.a_key = np.ones(T, dtype=np.uint64)
        st.a_stats = np.zeros((T, 0))
        st.a_sib = np.full(T, -1, dtype=np.int64)
        st.a_parent = np.full(T, -1, dtype=np.int64)
        st.prev_hist = None  # [A_prev, d, B, k] histograms of last level's split nodes
        st.rs_on = False     # this pass reduce-scatters its level histograms by feature (RS_MIN_BYTES)
        st.root_ids = [None] * T
        st.deep_rec = False  # set at the switch to node ids (deep_switch)
        st.wdeep = None
        st.node_count = st.forest.num_nodes
        return st

    def _fit_rows(self, st: "_FitState", codes_pre) -> None:
        """The fit's row state: a node permutation (one tree, segment mode), u16 row codes (+ the fixed-point
        scales every rank agrees on), or int32 node ids."""
        data, dev, n, T = self.data, self.device, self.data.n_local, st.T
        stats_rows, weights = st.stats_rows, st.weights
        st.codes = st.node = st.perm = None
        st.wmax = 1
        st.lazy_codes = None  # a lazy K.BootstrapCodes: the level-0 root histogram draws the codes
        if st.use_seg:
            w1 = None if weights is None else weights.reshape(-1)
            st.wmax = int(w1.max().item()) if (w1 is not None and w1.numel()) else 1
            perm = (torch.arange(n, dtype=torch.int32, device=dev) if w1 is None else
                    torch.nonzero(w1 > 0).flatten().to(torch.int32))
            pl = perm.long()
            st.perm = perm
            st.v1p = stats_rows["v1"].float()[pl].contiguous()
            st.v0p = None if stats_rows.get("v0") is None else stats_rows["v0"].float()[pl].contiguous()
            st.wp = None if (w1 is None or st.wmax <= 1) else w1[pl].to(torch.uint8).contiguous()
            # scales agreed over all ranks (max |v|, max weight, global row count): the int64 fixed-point
            # level histograms all-reduce exactly, so the tree does not depend on the GPU count
            st.seg_scales = K.seg_scales(st.v0p, st.v1p, st.wmax, data.n_global, self.comm)
            st.seg_raw = st.seg_scales if st.v0p is not None else st.seg_scales[1]
            st.segs = np.array([[0, perm.numel()]], dtype=np.int64)
        elif st.use_codes:
            if codes_pre is not None:
                st.codes, st.wmax = codes_pre.codes, codes_pre.wmax()
                if getattr(codes_pre, "pending", False):
                    st.lazy_codes = codes_pre
            else:
                st.codes, st.wmax = K.codes_init_max(weights, T, n, dev)
            if st.use_mseg:
                # one quantisation scale for every rank: the int64 level histograms then all-reduce to
                # the same sums on 1 or N GPUs (the forest does not depend on the GPU count)
                v0s = stats_rows.get("v0")
                st.mseg_scales = (1.0, 1.0) if (st.cls2 or st.cls3) else \
                    K.seg_scales(None if v0s is None else v0s.float(), stats_rows["v1"].float(), st.wmax,
                                 data.n_global, self.comm)
                st.mseg_raw = st.mseg_scales[1] if v0s is None else st.mseg_scales
        else:
            st.node = torch.arange(T, dtype=torch.int32, device=dev)[:, None].expand(T, n).contiguous() if n else \
                torch.zeros((T, 0), dtype=torch.int32, device=dev)

    def _fit_finish(self, st: "_FitState") -> Forest:
        forest = st.forest
        # the last level's bookkeeping stays with the forest (settled by the predictor right after its launch, or
        # by the first reader of the node lists)
        forest._pending.extend(st.pending)
        st.pending.clear()
        forest.roots.extend(st.root_ids)
        forest._dev = {}
        if st.heap_dev is not None:
            # the device heap of a deferred last level (the host arrays follow when the pending work runs)
            forest._dev[("heap", str(self.device), "value")] = st.heap_dev
        elif st.heap is not None:
            self._heap_to_forest(st)
        return forest

    @staticmethod
    def _heap_to_forest(st: "_FitState") -> None:
        S_ = 2 ** (st.heap_depth + 1) - 1
        st.forest._heap_np = (np.ascontiguousarray(st.heap[:, :S_]), np.ascontiguousarray(st.heap_v[:, :S_]),
                              st.heap_depth)

    def _defer_last_ok(self, st: "_FitState", depth: int) -> bool:
        """The last split level of a regression forest whose predict heap the trainer fills: decided on the device
        (K.heap_last_level) with its host side deferred (HEAP_LAST_DEVICE)."""
        p = self.p
        return (HEAP_LAST_DEVICE and st.heap is not None and depth > 0 and depth + 1 >= p.max_depth and
                not self.classification and p.impurity != "xgb" and not st.margin_ok and
                not self.data.categorical and not self.data.missing_bin)

    def _defer_decisions(self, st: "_FitState", lv: "_Level", src: torch.Tensor, depth: int) -> None:
        """Queue the last level's decisions into a device copy of the predict heap and their copy to the host;
        ``_level_deferred`` finishes the level on the host later."""
        dev = self.device
        D = depth + 1
        S_ = 2 ** (D + 1) - 1
        heap_np = K.pack_heap(st.heap[:, :S_], st.heap_v[:, :S_], D)
        A = len(st.a_tree)
        h_t, m_t, at, ak, aw = K.upload(dev, heap_np, np.zeros(8, np.int32), st.a_tree.astype(np.int32),
                                        st.a_key.astype(np.int32), self._weights_v(st.a_stats).astype(np.float64))
        thr = getattr(self, "_thr32", None)
        if thr is None or thr.device != h_t.device:
            thr, = K.upload(dev, np.ascontiguousarray(self.data.thresholds, dtype=np.float32))
            self._thr32 = thr
        assert src.shape[0] == A
        K.heap_last_level(src, at, ak, aw, thr, self.p.min_info_gain, 2.0 * self.p.min_instances, h_t, D)
        st.heap_dev = (h_t, D, m_t)
        host_p = torch.empty(src.shape, dtype=src.dtype, pin_memory=dev.type == "cuda")
        host_p.copy_(src, non_blocking=True)
        ev = None
        if dev.type == "cuda":
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
        lv.deferred = (host_p, ev)

    def _level_deferred(self, st: "_FitState", lv: "_Level", depth: int) -> None:
        """The host side of a deferred last level (forest pending work): the decisions, the node lists, the heap
        arrays."""
        host_p, ev = lv.deferred
        if ev is not None:
            ev.synchronize()
        host = host_p.numpy()
        lv.lst_h, lv.rst_h = host[:, 3:5], host[:, 5:7]
        lv.mr_h = None
        lv.gain_h, lv.bf_h, lv.bb_h = host[:, 0], host[:, 1].astype(np.int64), host[:, 2].astype(np.int64)
        lv.order_h = None
        self._level_advance(st, lv, depth)
        st.flush()
        if st.heap is not None:
            self._heap_to_forest(st)

    # ------------------------------------------------------------ level: tables
    def _level_tables(self, st: "_FitState", depth: int) -> "_Level":
        """Which active nodes build a histogram (the smaller of two siblings), the level's feature masks and its
        small device tables (one host -> device copy)."""
        p, data, dev, d, T = self.p, self.data, self.device, self.data.d, st.T
        lv = _Level()
        A = len(st.a_tree)
        lv.A = A
        lv.build = np.ones(A, dtype=bool)
        if depth > 0:
            lv.build = _built_nodes(self._weights_v(st.a_stats), st.a_sib, st.a_parent)
        lv.build_ids = np.nonzero(lv.build)[0]
        lv.slot_of = np.full(A, -1, dtype=np.int32)
        lv.slot_of[lv.build_ids] = np.arange(len(lv.build_ids), dtype=np.int32)
        lv.slot_tree = st.a_tree[lv.build_ids]
        lv.masks_np = None
        lv.masks_dev = None  # the same words drawn on the GPU (no host consumer this level)
        mask_base = None
        lv.tid = None
        if st.need_masks:
            lv.tid = st.a_tree if p.tree_ids is None else np.asarray(p.tree_ids, dtype=np.int64)[st.a_tree]
            if MASKS_DEV and dev.type == "cuda" and \
                    d <= K.FEATURE_MASKS_MAX_D and p.feature_subset is not None and 0 < p.feature_subset < d:
                mask_base = self._mask_base(lv.tid.astype(np.uint64), st.a_key)
            else:
                lv.masks_np = self._feature_masks(lv.tid.astype(np.uint64), st.a_key)
        lv.tfirst = torch.from_numpy(np.searchsorted(st.a_tree, np.arange(T), side="left").astype(np.int32))
        # the level's small device tables in ONE host->device copy (each separate copy was a blit kernel plus a
        # launch gap): hist_assemble's (slot, parent, sibling), the decode's a_tree / tfirst, the mask bases
        lv.lvl = None
        if dev.type == "cuda":
            lv.lvl = K.upload(dev, K.assemble_table(lv.slot_of, st.a_parent, st.a_sib), st.a_tree.astype(np.int32),
                              lv.tfirst.numpy().astype(np.int32),
                              *([mask_base.view(np.int64)] if mask_base is not None else []))
            if mask_base is not None:
                lv.masks_dev = K.feature_masks(mask_base, d, p.feature_subset, dev, base_dev=lv.lvl[3])
        return lv

    # ------------------------------------------------------------ level: histograms
    def _root_rows(self):
        """Row-major bins for the histograms straight from the codes: seg10 rows (B <= 40) or standard rows
        (boosting, 80 < B <= 256), else None."""
        data = self.data
        if self.device.type == "cuda" and ROOT_HIST:
            if data.bins_s10 is not None and data.d <= 100 and data.B <= 40:
                return data.bins_s10
            if 80 < data.B <= 256 and data.bins_rm is not None:
                return data.bins_rm
        return None

    def _level_histogram(self, st: "_FitState", lv: "_Level", depth: int) -> None:
        """lv.Hb: the level's built-slot histograms (int64 fixed-point sums on the record / segment paths, their
        scale in lv.hist_raw_scale; lv.reduced when they are already summed over ranks)."""
        data, dev, d, B, T = self.data, self.device, self.data.d, self.data.B, st.T
        stats_rows, wmax = st.stats_rows, st.wmax
        build_ids, slot_of, slot_tree, tfirst = lv.build_ids, lv.slot_of, lv.slot_tree, lv.tfirst
        S = len(build_ids)
        lv.hist_raw_scale = None
        lv.reduced = False
        # levels with <= 1 built node per tree (0: the roots, 1: the smaller children): the records are compacted
        # inside the histogram kernel (no codes_compact pass)
        root_rows = self._root_rows()
        root_ok = (root_rows is not None and st.use_mseg and (depth >= 1 or MSEG_L0) and st.rec_ok and
                   S > 0 and np.bincount(slot_tree, minlength=T).max() <= 1)
        draw = None
        if st.lazy_codes is not None:
            # the bootstrap draws are still pending: the level-0 root histogram (seg10 rows) draws and writes the
            # codes itself, any other path materialises them first
            if depth == 0 and root_ok and root_rows is data.bins_s10 and K.POISSON_FUSED and S == T:
                draw = st.lazy_codes.draw_args()
            else:
                st.lazy_codes.materialize()
            st.lazy_codes.mark_drawn()
            st.lazy_codes = None
        if root_ok:
            sl_node = build_ids - tfirst.numpy()[slot_tree]  # the slot's local node in its tree's codes
            # one launch for every slot, then the level's one all-reduce: these levels hold one node per
            # tree (20 x 100 x 40 cells = 1.3 MB at the headline), too little to overlap, and slot chunks
            # of a 1.25e7-row shard would launch ~1 round of blocks each (half of it idle)
            lv.Hb = K.seg_hist_codes(root_rows, d, B, st.codes, stats_rows["v1"], st.mseg_scales[1], wmax,
                                     slot_tree, sl_node, 0, S,
                                     torch.zeros((S, d, B, K.hist_cols(st.cls3)), dtype=torch.int64, device=dev),
                                     draw=draw, cls3=st.cls3)
            lv.hist_raw_scale = st.mseg_raw
        elif st.use_mseg and (depth >= 1 or MSEG_L0):
            # gather the rows of the built nodes into slot segments, then segment histograms of packed
            # item records on every device (the CPU emulates the HIP compaction + flat histogram
            # exactly, so gloo ranks traverse the integer path RCCL ranks take)
            perm, v0p, v1p, wp, sg = K.codes_compact(st.codes, tfirst, slot_of, S, stats_rows.get("v0"),
                                                     stats_rows["v1"],
                                                     rec_scale=st.mseg_scales[1] if st.rec_ok else None)
            is_rec = st.rec_ok and v1p is None
            sb = np.concatenate([sg, np.arange(S, dtype=np.int64)[:, None]], 1)
            lv_bytes = S * d * B * K.hist_cols(st.cls3) * 8
            if is_rec and (self.comm.distributed or HIST_OVERLAP_FORCE) and HIST_OVERLAP > 1 and S >= 2 and \
                    lv_bytes >= HIST_OVERLAP_MIN_BYTES:
                # comm/compute overlap: the level's slots are built in chunks, each chunk's int64 histogram
                # all-reduced -- or, on reduce-scatter levels, reduce-scattered by feature -- asynchronously on
                # the RCCL stream while the next chunk is built
                rs = self._rs_level(lv_bytes, st.rs_on)
                res = self._hist_overlapped(data, d, B, perm, sb, S, wmax, st.mseg_scales, dev, cls3=st.cls3,
                                            rs=rs)
                if rs:
                    lv.Hb, lv.rs_slice = res
                    self._rs_enter(st, lv.rs_slice)
                else:
                    lv.Hb = res
                lv.reduced = True
            else:
                rm, s10 = (data.record_rows() if is_rec else (data.row_major_bins(), False)) \
                    if dev.type == "cuda" else (None, False)
                lv.Hb = K.seg_hist(data.bins, d, B, perm, v0p, v1p, wp, sb, S, wmax, st.mseg_scales, bins_rm=rm,
                                   interleave=True, rec=is_rec, raw=True, rm_s10=s10, cls3=st.cls3)
            lv.hist_raw_scale = st.mseg_raw
        elif st.deep_rec and S and np.bincount(st.a_tree, minlength=T).max() <= K.NODE_COMPACT_MAX_LOC:
            # levels below the u16 codes (binary classification deeper than 8): the built rows' packed
            # records from the node ids, then the same record histograms as the shallow levels (the
            # node-id kernel re-read every row once per LDS-sized slot group: ~290 ms per level at
            # 1e7 rows x 100 trees)
            perm, sg = K.node_compact(st.node, st.wdeep, tfirst.numpy(), slot_of, S, stats_rows["v1"],
                                      st.mseg_scales[1])
            sb = np.concatenate([sg, np.arange(S, dtype=np.int64)[:, None]], 1)
            rm, s10 = data.record_rows() if dev.type == "cuda" else (None, False)
            lv.Hb = K.seg_hist(data.bins, d, B, perm, None, None, None, sb, S, wmax, st.mseg_scales, bins_rm=rm,
                               interleave=True, rec=True, raw=True, rm_s10=s10)
            lv.hist_raw_scale = st.mseg_raw
        elif st.use_seg:
            sb = np.stack([st.segs[build_ids, 0], st.segs[build_ids, 1], slot_of[build_ids].astype(np.int64)], 1)
            lv.Hb = K.seg_hist(data.bins, d, B, st.perm, st.v0p, st.v1p, st.wp, sb, S, wmax, st.seg_scales,
                               # sparse node segments (>= 4 built nodes) gather whole rows from the
                               # row-major copy; dense shallow levels stream the [G][n] layout
                               bins_rm=data.row_major_bins() if (K.SEG_ROW_MAJOR and dev.type == "cuda"
                                                                 and S >= 4) else None,
                               interleave=st.use_mseg, raw=True)
            lv.hist_raw_scale = st.seg_raw
        elif st.use_codes:
            lv.Hb = K.hist_codes(1 if self.classification else 0, data.bins, d, st.codes, tfirst,
                                 stats_rows.get("v0"), stats_rows.get("v1"), stats_rows.get("label"), self.C,
                                 K.upload(dev, slot_of)[0], slot_tree, st.a_tree, None, B, wmax=wmax)
        elif self.classification:
            lv.Hb = K.hist_classes(data.bins, d, st.node, st.weights, stats_rows["label"], self.C,
                                   K.upload(dev, slot_of)[0], slot_tree, None, B, id_tree=st.a_tree)
        else:
            lv.Hb = K.hist_moments(data.bins, d, st.node, st.weights, stats_rows.get("v0"), stats_rows["v1"],
                                   K.upload(dev, slot_of)[0], slot_tree, None, B, id_tree=st.a_tree)
        if st.cls2 and lv.hist_raw_scale is not None:
            lv.Hb[..., 0] -= lv.Hb[..., 1]  # packed (W, W1) -> class counts (W0, W1), exact int64
        elif st.cls3 and lv.hist_raw_scale is not None:
            lv.Hb = K.cls3_expand(lv.Hb)  # (W, W1, W2) -> class counts (W0, W1, W2)

    def _level_reduce(self, st: "_FitState", lv: "_Level") -> None:
        """The level histograms summed over ranks: one fused all-reduce, or (large int64 levels) a reduce-scatter
        by feature -- lv.rs_slice is then this rank's feature range and prev_hist is cut to it."""
        if lv.reduced:
            return
        if self._rs_want(lv.Hb, st.rs_on):
            lv.rs_slice, lv.Hb = self._reduce_scatter_features(lv.Hb, self.data.d)
            self._rs_enter(st, lv.rs_slice)
        else:
            with _tr.span("tree.allreduce", cat="comm", bytes=lv.Hb.numel() * 8):
                self.comm.all_reduce(lv.Hb)  # one fused RCCL all-reduce per level

    # ------------------------------------------------------------ level: split decisions
    def _level_decide(self, st: "_FitState", lv: "_Level", depth: int) -> None:
        """Assemble every active node's histogram, find the best splits (K6 kernels on the GPU), queue the device
        decode + partition behind them where it applies, and bring the decisions to the host (lv.gain_h,
        lv.bf_h, lv.bb_h, lv.lst_h, lv.rst_h, lv.mr_h, lv.catm_h, lv.order_h, lv.cat_feats; level 0 also sets the
        roots' stats)."""
        p, dev, d, T = self.p, self.device, self.data.d, st.T
        Hb = lv.Hb
        derived = np.nonzero(~lv.build)[0]
        is_raw = Hb.dtype == torch.int64
        if is_raw or len(derived):
            # one kernel (CPU: the same arithmetic in torch): fixed-point -> fp64 and parent - sibling
            H = K.hist_assemble(Hb, lv.hist_raw_scale if is_raw else None, st.prev_hist if len(derived) else None,
                                lv.slot_of, st.a_parent, st.a_sib, table=lv.lvl[0] if lv.lvl is not None else None)
        else:
            H = Hb
        lv.H = H
        masks_t = lv.masks_dev if lv.masks_dev is not None else \
            (K.upload(dev, lv.masks_np.view(np.int32))[0] if lv.masks_np is not None else None)
        lv.catm_h = None  # left-category bit masks of the native categorical scan
        lv.dec = None     # device-decoded partition tables (partition already queued)
        lv.deferred = None  # (pinned decisions, event): the last level decided on the device (_defer_decisions)
        defer = self._defer_last_ok(st, depth)
        order = None
        lv.cat_feats = []
        pre = (lv.lvl[1], lv.lvl[2]) if lv.lvl is not None else None
        # (deep forests: not at the level that leaves the codes for node ids; below it on the node ids)
        deep_ids = st.deep_switch and st.node is not None
        leaving_codes = st.deep_switch and st.use_codes and depth + 1 >= 8
        if lv.rs_slice is not None or self._native_split(dev):
            # K6 in one kernel: node totals, prefix scans, gains, masks, argmax
            mb = p.impurity == "xgb" and self.data.missing_bin
            if lv.rs_slice is not None:
                masks_np = lv.masks_np
                if lv.masks_dev is not None:
                    masks_np = self._feature_masks(lv.tid.astype(np.uint64), st.a_key)
                so, tot = self._rs_split(H, lv.rs_slice, masks_np, d, dev, exact=self._k6_exact(st, lv))
            else:
                so, tot = K.split_scan(H, self._nthr_dev(dev), masks_t, 1 if p.impurity == "xgb" else 0,
                                       p.min_instances, p.reg_lambda, p.gamma, p.min_child_weight, missing_bin=mb,
                                       exact=self._k6_exact(st, lv))
            host_p = None
            if self._device_decode_ok(dev, st.use_codes or deep_ids, mb) and \
                    (depth + 1 < p.max_depth or st.margin_ok) and not leaving_codes:
                # the decisions leave for the host first (pinned, async): they arrive while the partition runs
                src = torch.cat([so, tot], 1) if depth == 0 else so
                host_p = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
                host_p.copy_(src, non_blocking=True)
                host_ev = torch.cuda.Event()
                host_ev.record(torch.cuda.current_stream(dev))
                # the partition tables decoded on the device and the row partition queued right behind K6:
                # the GPU partitions while the decisions travel to the host and the host builds the forest
                # and the next level's layout (the same decode on the host, checked in the checked build)
                lv.dec = self._device_partition(so, tot, st.a_tree, lv.tfirst, T, depth, mb, st.codes,
                                                margin=st.margin if st.margin_ok else None,
                                                node=st.node if deep_ids else None, pre=pre)
            # so [A, 8] = gain, feature, bin, left (2), right (2), missing-goes-right: copied to the host as is
            # (plus the node totals at level 0), no per-column device ops
            sw = so.shape[1]
            if host_p is None and defer:
                self._defer_decisions(st, lv, so, depth)
                st.flush()
                return
            st.flush()  # the previous level's forest bookkeeping, while the GPU runs this level's kernels
            if host_p is not None:
                host_ev.synchronize()
                host = host_p.numpy()
            else:
                host = (torch.cat([so, tot], 1) if depth == 0 else so).cpu().numpy()
            lv.lst_h, lv.rst_h = host[:, 3:5], host[:, 5:7]
            lv.mr_h = host[:, 7] > 0.5 if mb else None
            if depth == 0:
                st.a_stats = host[:, sw:sw + tot.shape[1]].copy()
        elif self._native_split_ex(dev):
            # classification / categorical K6 in one kernel (centroid-ordered categories, Gini / entropy)
            so, tot, cm = K.split_scan_ex(H, self._nthr_dev(dev), masks_t, p.impurity, p.min_instances)
            kk = tot.shape[1]
            src = torch.cat([so, cm.double()] + ([tot] if depth == 0 else []), 1)
            reg_ex = not self.classification and kk == 2  # variance regression with categorical features
            if (st.cls2 or reg_ex) and (st.use_codes or deep_ids) and DEVICE_DECODE and depth + 1 < p.max_depth \
                    and not leaving_codes:
                # binary classification / categorical regression on the codes: the same device decode +
                # partition as numeric regression, queued behind K6 while the decisions travel to the host;
                # categorical winners split by K6's category bitmasks.  The decode reads (gain, feature, bin,
                # left weight, ., right weight, .); a pure child (one class) weighs 0 there, so it is a leaf on
                # the device exactly as on the host
                host_p = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
                host_p.copy_(src, non_blocking=True)
                host_ev = torch.cuda.Event()
                host_ev.record(torch.cuda.current_stream(dev))
                if st.cls2:
                    l0, l1, r0, r1 = so[:, 4], so[:, 5], so[:, 6], so[:, 7]
                    zero = torch.zeros_like(l0)
                    so_d = torch.stack([so[:, 0], so[:, 1], so[:, 2],
                                        torch.where((l0 > 0) & (l1 > 0), l0 + l1, zero), l1,
                                        torch.where((r0 > 0) & (r1 > 0), r0 + r1, zero), r1], 1)
                    tot_d = tot.sum(1, keepdim=True)
                else:
                    so_d = so[:, [0, 1, 2, 4, 5, 6, 7]]
                    tot_d = tot
                lv.dec = self._device_partition(so_d, tot_d, st.a_tree, lv.tfirst, T, depth, False, st.codes,
                                                catm=cm if self.data.categorical else None,
                                                node=st.node if deep_ids else None, pre=pre)
                st.flush()
                host_ev.synchronize()
                host = host_p.numpy()
            else:
                st.flush()
                host = src.cpu().numpy()
            lv.lst_h, lv.rst_h = host[:, 4:4 + kk], host[:, 4 + kk:4 + 2 * kk]
            c0 = 4 + 2 * kk
            lv.catm_h = (host[:, c0:c0 + 8].astype(np.int64) & 0xFFFFFFFF).astype(np.uint32)
            lv.mr_h = None
            if depth == 0:
                st.a_stats = host[:, c0 + 8:c0 + 8 + kk].copy()
        else:
            tot = self._node_stats(H, None)
            gain, bf, bb, lst, rst, order, lv.cat_feats, miss_right = self._best_splits(H, tot, masks_t)
            # one device->host transfer for the whole level's decisions (ids < 2^53 are exact in f64)
            kk = lst.shape[1]
            cols = [gain[:, None], bf[:, None].double(), bb[:, None].double(), lst, rst]
            if miss_right is not None:
                cols.append(miss_right[:, None].double())
            if depth == 0:
                cols.append(tot)
            if defer and kk == 2 and order is None:
                self._defer_decisions(st, lv, torch.cat(cols, 1), depth)
                st.flush()
                return
            st.flush()
            host = torch.cat(cols, 1).cpu().numpy()
            lv.lst_h, lv.rst_h = host[:, 3:3 + kk], host[:, 3 + kk:3 + 2 * kk]
            c0 = 3 + 2 * kk
            lv.mr_h = None
            if miss_right is not None:
                lv.mr_h = host[:, c0] != 0
                c0 += 1
            if depth == 0:
                st.a_stats = host[:, c0:c0 + tot.shape[1]].copy()
        lv.gain_h, lv.bf_h, lv.bb_h = host[:, 0], host[:, 1].astype(np.int64), host[:, 2].astype(np.int64)
        lv.order_h = order.cpu().numpy() if order is not None else None

    # ------------------------------------------------------------ level: children and bookkeeping
    def _level_advance(self, st: "_FitState", lv: "_Level", depth: int) -> None:
        """The level's splits on the host: the children (the next active set), the row partition where the device
        did not already queue it, and the forest / heap bookkeeping (deferred to the next level's sync)."""
        p, data, dev, T, A = self.p, self.data, self.device, st.T, lv.A
        forest = st.forest
        a_tree, a_fid, a_key = st.a_tree, st.a_fid, st.a_key
        if depth == 0:
            a_fid = st.a_fid = forest.add_many(self._leaf_values_v(st.a_stats), self._weights_v(st.a_stats), depth,
                                               self._impurities_v(st.a_stats))
            st.node_count = forest.num_nodes
            if st.heap is not None:
                st.heap_v[a_tree, 0] = self._leaf_values_v(st.a_stats)[:, 0]
            for t_, fid_ in zip(a_tree.tolist(), a_fid.tolist()):
                st.root_ids[t_] = fid_
        gain_h, bf_h, bb_h, mr_h, catm_h = lv.gain_h, lv.bf_h, lv.bb_h, lv.mr_h, lv.catm_h
        W_a = self._weights_v(st.a_stats)
        with np.errstate(invalid="ignore"):
            can = np.isfinite(gain_h) & (gain_h > 0) & (gain_h >= p.min_info_gain) & (W_a >= 2 * p.min_instances)
        if depth >= p.max_depth:
            can[:] = False
        sp = np.nonzero(can)[0]
        split_feat = np.full(A, -1, dtype=np.int32)
        split_bin = np.zeros(A, dtype=np.int32)
        cat_off = np.full(A, -1, dtype=np.int32)
        cat_masks = []
        child = np.full(2 * A, -1, dtype=np.int32)
        f_sp, b_sp, fid_sp = bf_h[sp], bb_h[sp], a_fid[sp]
        thr_sp = np.zeros(len(sp))
        plain = np.ones(len(sp), dtype=bool)
        if data.categorical or mr_h is not None:
            st.flush()  # the writes below address the nodes the previous level appended
            for j, a in enumerate(sp.tolist()):
                f, b = int(f_sp[j]), int(b_sp[j])
                if f in data.categorical:
                    if catm_h is not None:
                        m = catm_h[a].copy()
                    else:
                        ci = lv.cat_feats.index(f)
                        m = np.zeros(8, dtype=np.uint32)
                        for c in lv.order_h[a, ci, : b + 1]:
                            m[int(c) >> 5] |= np.uint32(1) << np.uint32(int(c) & 31)
                elif mr_h is not None and mr_h[a]:
                    # missing (bin 0) goes right: left = bins 1..b, expressed as a bin-set split
                    m = np.zeros(8, dtype=np.uint32)
                    for c in range(1, b + 1):
                        m[c >> 5] |= np.uint32(1) << np.uint32(c & 31)
                    forest.bin[int(fid_sp[j])] = b
                    thr_sp[j] = float(data.thresholds[f, b])
                else:
                    continue
                plain[j] = False
                forest.is_cat[int(fid_sp[j])] = True
                forest.catmask[int(fid_sp[j])] = m
                cat_off[a] = len(cat_masks)
                cat_masks.append(m)
        cat_f = np.array([f in data.categorical for f in f_sp.tolist()], dtype=bool) if \
            data.categorical else np.zeros(len(sp), dtype=bool)
        num = ~cat_f  # numeric splits carry a bin threshold (missing-right ones too)
        if num.any():
            thr_sp[num] = data.thresholds[f_sp[num], b_sp[num]]
        split_bin[sp[plain]] = b_sp[plain]
        split_feat[sp] = f_sp
        # children in (node, side) order: ids base + 2j (left), base + 2j + 1 (right)
        k_st = lv.lst_h.shape[1]
        ch_st = np.stack([lv.lst_h[sp], lv.rst_h[sp]], 1).reshape(-1, k_st)
        # forest ids of the children (appended after the partition launch: the forest bookkeeping then
        # runs on the host while the GPU partitions the rows)
        ch_ids = np.arange(st.node_count, st.node_count + 2 * len(sp), dtype=np.int64)
        st.node_count += 2 * len(sp)
        cw = self._weights_v(ch_st)
        leaf = (cw < 2 * p.min_instances) | (depth + 1 >= p.max_depth)
        if self.classification:
            leaf |= (ch_st > 0).sum(1) <= 1  # pure node
        nl = np.nonzero(~leaf)[0]
        ch_par = np.repeat(sp, 2)
        child[2 * ch_par[nl] + (nl & 1)] = np.arange(len(nl), dtype=np.int32)
        n_tree = a_tree[ch_par[nl]]
        n_fid = ch_ids[nl]
        n_key = a_key[ch_par[nl]] * np.uint64(2) + (nl & 1).astype(np.uint64)
        n_stats = ch_st[nl]
        n_parent = ch_par[nl].astype(np.int64)
        # siblings (both children active) for subtraction; a single active child is built directly
        pos = np.full(2 * len(sp), -1, dtype=np.int64)
        pos[nl] = np.arange(len(nl))
        lp, rp = pos[0::2], pos[1::2]
        both = (lp >= 0) & (rp >= 0)
        n_sib = np.full(len(nl), -1, dtype=np.int64)
        n_sib[lp[both]] = rp[both]
        n_sib[rp[both]] = lp[both]
        n_parent[n_sib < 0] = -1
        if len(nl) and st.deep_switch and st.use_codes and depth + 1 >= 8:
            # the next level can hold more than 255 nodes per tree: leave the u16 codes for node ids
            # (active index of the node, -1 = done), partitioned and histogrammed by the node-id kernels
            node, st.wdeep = K.decode_codes(st.codes, lv.tfirst)  # host tfirst: uploaded once, no D2H
            st.node = node.contiguous()
            # the node-id histogram kernels (levels past NODE_COMPACT_MAX_LOC nodes per tree) read the row weights
            # from ``weights``: None when the bootstrap draws arrived as row codes (BootstrapCodes)
            st.weights = st.wdeep
            # below level 8 the record histograms continue from the node ids (K.node_compact)
            st.deep_rec = st.use_mseg and st.rec_ok
            st.use_codes = st.use_mseg = False
            st.codes = None
        if len(nl):
            cm = np.stack(cat_masks).view(np.int32) if cat_masks else np.zeros((0, 8), np.int32)
            with _tr.span("tree.partition", depth=depth):
                if st.use_seg:
                    st.perm, st.v0p, st.v1p, st.wp, st.segs = K.seg_partition(
                        data.bins, st.perm, st.v0p, st.v1p, st.wp, st.segs, split_feat, split_bin, cat_off,
                        cm.reshape(-1), child, len(nl))
                elif lv.dec is not None:  # partitioned on the device behind K6
                    if K._lib.DEBUG:
                        self._check_decode(lv.dec, split_feat, split_bin, cat_off, cat_masks, child, n_tree, T)
                elif st.use_codes:
                    tfirst_next = torch.from_numpy(np.searchsorted(n_tree, np.arange(T), side="left").astype(np.int32))
                    K.partition_codes(data.bins, st.codes, lv.tfirst, tfirst_next, torch.from_numpy(split_feat),
                                      torch.from_numpy(split_bin), torch.from_numpy(cat_off),
                                      torch.from_numpy(cm.reshape(-1)), torch.from_numpy(child))
                else:
                    K.partition(data.bins, st.node, *K.upload(dev, split_feat, split_bin, cat_off, cm.reshape(-1),
                                                              child))
        ch_vals = self._leaf_values_v(ch_st)
        # the forest's node lists for this level are appended and split at the next level's decision sync
        # (flush), i.e. while the GPU runs that level's histogram / K6 / partition, not between this level's
        # decisions and the next level's launches (~0.2-0.4 ms of numpy per level at the headline's widths)
        st.pending.append(functools.partial(_forest_level_ops, forest, (ch_vals, cw, depth + 1,
                                                                         self._impurities_v(ch_st)),
                                            (fid_sp, f_sp, gain_h[sp], b_sp, thr_sp, num, ch_ids[0::2],
                                             ch_ids[1::2]), ch_ids[0] if len(ch_ids) else None, len(ch_ids)))
        if st.heap is not None and len(sp):
            if not plain.all():
                st.heap = None  # bin-set splits: Forest.heap_arrays builds the table from the forest
            else:
                tsp, ksp = a_tree[sp], a_key[sp].astype(np.int64)
                st.heap[tsp, ksp - 1, 0] = f_sp
                st.heap[tsp, ksp - 1, 1] = thr_sp.astype(np.float32).view(np.int32)
                ck = np.stack([2 * ksp, 2 * ksp + 1], 1).reshape(-1)
                st.heap_v[np.repeat(tsp, 2), ck - 1] = ch_vals[:, 0]
                st.heap_depth = depth + 1
        st.prev_hist = lv.H
        st.a_tree, st.a_fid, st.a_key, st.a_stats, st.a_sib, st.a_parent = \
            n_tree, n_fid, n_key, n_stats, n_sib, n_parent


class _FitState:
    """Per-fit state of ForestTrainer.train: the paths chosen once per fit (``_fit_paths``), the row state
    (``_fit_rows``: codes / node ids / segment permutation and their fixed-point scales), the active node set as
    host arrays (a_tree, a_fid, a_key, a_stats, a_sib, a_parent), the previous level's histograms, the forest and
    its predict heap table, and the forest bookkeeping deferred to the next level's sync (``pending``)."""

    def __init__(self):
        self.pending = []

    def flush(self) -> None:
        """Run the deferred forest bookkeeping of the previous level (called while the GPU runs this level)."""
        while self.pending:
            self.pending.pop(0)()


class _Level:
    """One level's tables (``_level_tables``), histograms (``_level_histogram`` / ``_level_reduce``) and host-side
    decisions (``_level_decide``)."""
    rs_slice = None   # (f0, f1): this rank's feature range once the level was reduce-scattered by feature
    reduced = False


from ...ops import tune as _tune  # noqa: E402  (CDNAML_TUNE overrides of the constants above)
_tune.apply(__import__(__name__, fromlist=["_"]))
_tune.check()
